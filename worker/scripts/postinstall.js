#!/usr/bin/env node
// npm postinstall for the gpu-worker launcher: report what the worker will run on.
// Never fails the install — it only prints hints (Python version, ROCm stack, MI355X GPUs).
'use strict';
const { spawnSync } = require('child_process');
const fs = require('fs');

function run(cmd, args) {
  try {
    const r = spawnSync(cmd, args, { encoding: 'utf8', timeout: 10000 });
    return r.status === 0 ? (r.stdout || '').trim() : null;
  } catch (e) {
    return null;
  }
}

function findPython() {
  for (const exe of ['python3', 'python', 'py']) {
    const v = run(exe, ['-c', 'import sys;print("%d.%d" % sys.version_info[:2])']);
    if (!v) continue;
    const [maj, min] = v.split('.').map(Number);
    if (maj > 3 || (maj === 3 && min >= 9)) return { exe, version: v };
  }
  return null;
}

function rocmInfo() {
  const out = { rocm: null, gpus: [] };
  if (fs.existsSync('/opt/rocm/.info/version')) {
    out.rocm = fs.readFileSync('/opt/rocm/.info/version', 'utf8').trim();
  }
  const agents = run('rocminfo', []) || '';
  for (const m of agents.matchAll(/Name:\s+(gfx\w+)/g)) out.gpus.push(m[1]);
  return out;
}

const py = findPython();
const hw = rocmInfo();
console.log('\n[gpu-worker] installed');
console.log(py ? `  python  : ${py.exe} (${py.version})` : '  python  : NOT FOUND (need >= 3.9)');
console.log(hw.rocm ? `  rocm    : ${hw.rocm}` : '  rocm    : not detected (CPU / HF-only mode)');
if (hw.gpus.length) {
  const n950 = hw.gpus.filter((g) => g === 'gfx950').length;
  console.log(`  gpus    : ${hw.gpus.length} agent(s)${n950 ? `, ${n950} x MI355X (gfx950)` : ''}`);
}
console.log('  next    : gpu-worker install && gpu-worker configure && gpu-worker start\n');
