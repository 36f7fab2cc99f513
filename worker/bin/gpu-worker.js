#!/usr/bin/env node
// npm/npx launcher for the Python worker (reference worker/bin/gpu-worker.js).
// Dependency-free: finds a Python >= 3.9 (preferring ./.venv), checks that a ROCm
// PyTorch build is importable, then forwards all arguments to cli.py.
'use strict';
const { spawnSync, spawn } = require('child_process');
const fs = require('fs');
const path = require('path');

const PKG_DIR = path.resolve(__dirname, '..');

function pythonCandidates() {
  const venv = path.join(PKG_DIR, '.venv', process.platform === 'win32' ? 'Scripts/python.exe' : 'bin/python');
  const c = [];
  if (process.env.GPU_WORKER_PYTHON) c.push(process.env.GPU_WORKER_PYTHON);
  if (fs.existsSync(venv)) c.push(venv);
  return c.concat(['python3', 'python']);
}

function findPython() {
  for (const cmd of pythonCandidates()) {
    const r = spawnSync(cmd, ['-c', 'import sys; print("%d.%d" % sys.version_info[:2])'], { encoding: 'utf8' });
    if (r.status !== 0) continue;
    const [maj, min] = r.stdout.trim().split('.').map(Number);
    if (maj === 3 && min >= 9) return cmd;
  }
  return null;
}

function main() {
  const py = findPython();
  if (!py) {
    console.error('gpu-worker: Python >= 3.9 not found (set GPU_WORKER_PYTHON)');
    process.exit(1);
  }
  const args = process.argv.slice(2);
  if (args.length === 0) args.push('--help');
  if (args[0] === 'start') {
    const probe = spawnSync(py, ['-c', 'import torch; print(torch.version.hip or "")'], { encoding: 'utf8' });
    if (probe.status !== 0) {
      console.error('gpu-worker: PyTorch is not importable; install a ROCm build first');
      process.exit(1);
    }
    if (!probe.stdout.trim()) console.warn('gpu-worker: warning: PyTorch has no HIP runtime (CPU-only build)');
  }
  const child = spawn(py, [path.join(PKG_DIR, 'cli.py'), ...args], { stdio: 'inherit', cwd: process.cwd() });
  const forward = (sig) => () => child.kill(sig);
  process.on('SIGINT', forward('SIGINT'));
  process.on('SIGTERM', forward('SIGTERM'));
  child.on('exit', (code, signal) => process.exit(code === null ? (signal ? 1 : 0) : code));
}

main();
