#!/usr/bin/env node
// npm/npx launcher for the Python worker (behaviour of reference worker/bin/gpu-worker.js:
// first-run environment setup, dependency install, interactive menu, command forwarding).
//
// MI355X-first differences from the reference:
//  * ROCm, not CUDA: the PyTorch wheel index is chosen from the installed ROCm release
//    (/opt/rocm/.info/version, or `hipconfig --version`), and a ROCm PyTorch that the
//    system already has (the usual case on MI355X images) is reused through a
//    `--system-site-packages` venv instead of being downloaded again;
//  * offline clusters: GPU_WORKER_WHEELHOUSE=<dir> installs with --no-index from a local
//    wheel directory;
//  * after the Python deps, `cli.py install` builds the dgi HIP kernels for gfx950;
//  * no npm dependencies (no commander / inquirer / chalk / ora): argument parsing and
//    the menu are plain Node, so `npx gpu-worker` works without a registry.
// GPU_WORKER_DRY_RUN=1 prints the commands instead of running them (used by the tests).
'use strict';
const { spawnSync, spawn } = require('child_process');
const fs = require('fs');
const path = require('path');
const readline = require('readline');

const PKG_DIR = path.resolve(__dirname, '..');
const VENV = path.join(PKG_DIR, '.venv');
const VERSION = (() => {
  try { return JSON.parse(fs.readFileSync(path.join(PKG_DIR, 'package.json'), 'utf8')).version; } catch (e) { return '0.0.0'; }
})();
// ROCm releases with a PyTorch wheel index; a newer ROCm uses the newest index not above it
const ROCM_INDEXES = ['6.0', '6.1', '6.2', '6.3', '6.4', '7.0'];
const DRY = process.env.GPU_WORKER_DRY_RUN === '1';
const tty = process.stdout.isTTY;
const color = (c) => (s) => (tty ? `\x1b[${c}m${s}\x1b[0m` : String(s));
const red = color('31'), green = color('32'), yellow = color('33'), cyan = color('36'), bold = color('1');

// ------------------------------------------------------------------ probes
function probe(cmd, args) {
  try {
    const r = spawnSync(cmd, args, { encoding: 'utf8', timeout: 60000 });
    return r.status === 0 ? (r.stdout || '').trim() : null;
  } catch (e) {
    return null;
  }
}

function venvPython() {
  const p = path.join(VENV, process.platform === 'win32' ? 'Scripts/python.exe' : 'bin/python');
  return fs.existsSync(p) ? p : null;
}

function findPython() {
  const c = [];
  if (process.env.GPU_WORKER_PYTHON) c.push(process.env.GPU_WORKER_PYTHON);
  c.push('python3', 'python');
  for (const cmd of c) {
    const v = probe(cmd, ['-c', 'import sys; print("%d.%d" % sys.version_info[:2])']);
    if (!v) continue;
    const [maj, min] = v.split('.').map(Number);
    if (maj > 3 || (maj === 3 && min >= 9)) return cmd;
  }
  return null;
}

// ROCm release "major.minor" or null
function rocmVersion(env) {
  const e = env || process.env;
  if (e.GPU_WORKER_ROCM_VERSION) return e.GPU_WORKER_ROCM_VERSION;
  const root = e.ROCM_PATH || '/opt/rocm';
  try {
    const v = fs.readFileSync(path.join(root, '.info', 'version'), 'utf8').trim();
    const m = v.match(/^(\d+)\.(\d+)/);
    if (m) return `${m[1]}.${m[2]}`;
  } catch (err) { /* no ROCm install file */ }
  const h = probe('hipconfig', ['--version']);
  const m = h && h.match(/^(\d+)\.(\d+)/);
  return m ? `${m[1]}.${m[2]}` : null;
}

// PyTorch wheel index for a ROCm release (null: no ROCm, CPU wheels)
function torchIndexUrl(rocm) {
  if (!rocm) return null;
  const val = (v) => { const [a, b] = v.split('.').map(Number); return a * 100 + b; };
  let best = null;
  for (const v of ROCM_INDEXES) if (val(v) <= val(rocm)) best = v;
  return best ? `https://download.pytorch.org/whl/rocm${best}` : null;
}

// requirements.txt without torch lines (torch is installed separately, ROCm build)
function filterRequirements(text) {
  return text.split(/\r?\n/).filter((l) => {
    const t = l.trim();
    return !t || t.startsWith('#') || !/^torch(\s*[<>=!~].*)?$/.test(t);
  }).join('\n');
}

// 'hip' (ROCm torch importable), 'cpu' (torch without HIP), or null
function torchKind(py) {
  const out = probe(py, ['-c', 'import torch; print(torch.version.hip or "cpu")']);
  if (out === null) return null;
  return out === 'cpu' ? 'cpu' : 'hip';
}

// ------------------------------------------------------------------ actions
function run(cmd, args, opts) {
  const shown = [cmd].concat(args).map((a) => (/\s/.test(a) ? `"${a}"` : a)).join(' ');
  if (DRY) {
    console.log(`[dry-run] ${shown}`);
    return true;
  }
  console.log(cyan(`$ ${shown}`));
  const r = spawnSync(cmd, args, Object.assign({ stdio: 'inherit' }, opts || {}));
  return r.status === 0;
}

function createVenv(py, systemSite) {
  const args = ['-m', 'venv'];
  if (systemSite) args.push('--system-site-packages');
  args.push(VENV);
  if (!run(py, args)) {
    console.error(red('failed to create the virtual environment'));
    return false;
  }
  console.log(green(`virtual environment ready: ${VENV}${systemSite ? ' (reusing the system ROCm PyTorch)' : ''}`));
  return true;
}

// pip commands that install torch (ROCm wheels) + the worker requirements
function planInstall(py, env) {
  const e = env || process.env;
  const pip = [py, '-m', 'pip', 'install'];
  const house = e.GPU_WORKER_WHEELHOUSE;
  const src = house ? ['--no-index', '--find-links', house] : [];
  const steps = [];
  const kind = e.GPU_WORKER_TORCH_KIND !== undefined ? (e.GPU_WORKER_TORCH_KIND || null) : torchKind(py);
  if (kind !== 'hip') {
    const url = house ? null : torchIndexUrl(rocmVersion(e));
    steps.push(pip.concat(['torch'], src, url ? ['--index-url', url] : []));
  }
  const req = path.join(PKG_DIR, 'requirements.txt');
  if (fs.existsSync(req)) {
    const filtered = path.join(PKG_DIR, '.requirements.no-torch.txt');
    steps.push(pip.concat(['-r', filtered], src));
  }
  return { steps, torch: kind };
}

function installDependencies(py) {
  const plan = planInstall(py);
  if (plan.torch === 'hip') console.log(green('ROCm PyTorch already importable — not reinstalling torch'));
  else if (plan.torch === 'cpu') console.log(yellow('installed PyTorch has no HIP runtime — installing the ROCm build'));
  const req = path.join(PKG_DIR, 'requirements.txt');
  const filtered = path.join(PKG_DIR, '.requirements.no-torch.txt');
  if (fs.existsSync(req) && !DRY) fs.writeFileSync(filtered, filterRequirements(fs.readFileSync(req, 'utf8')));
  try {
    for (const s of plan.steps) {
      if (!run(s[0], s.slice(1))) {
        console.error(red('dependency installation failed'));
        return false;
      }
    }
  } finally {
    if (fs.existsSync(filtered)) fs.unlinkSync(filtered);
  }
  // build the gfx950 HIP kernels
  run(py, [path.join(PKG_DIR, 'cli.py'), 'install']);
  console.log(green('dependencies installed'));
  return true;
}

// one line reader for the whole session: piped answers ("2\n1\n") reach successive prompts
let lineQueue = null;
function closeInput() {
  if (lineQueue && lineQueue.rl) { lineQueue.rl.close(); lineQueue.rl = null; }
}
function ask(question) {
  if (lineQueue === null) {
    const rl = readline.createInterface({ input: process.stdin, terminal: false });
    lineQueue = { lines: [], waiters: [], closed: false, rl };
    rl.on('line', (l) => {
      const w = lineQueue.waiters.shift();
      if (w) w(l.trim()); else lineQueue.lines.push(l.trim());
    });
    rl.on('close', () => {
      lineQueue.closed = true;
      while (lineQueue.waiters.length) lineQueue.waiters.shift()('');
    });
  }
  process.stdout.write(question);
  if (lineQueue.lines.length) return Promise.resolve(lineQueue.lines.shift());
  if (lineQueue.closed) return Promise.resolve('');
  return new Promise((resolve) => lineQueue.waiters.push(resolve));
}

async function choose(title, choices) {
  console.log(bold(title));
  choices.forEach((c, i) => console.log(`  ${i + 1}) ${c.name}`));
  for (let tries = 0; tries < 3; tries++) {
    const a = await ask(`select [1-${choices.length}]: `);
    if (a === '') return choices[choices.length - 1].value;       // EOF / empty: last choice
    const n = Number(a);
    if (Number.isInteger(n) && n >= 1 && n <= choices.length) return choices[n - 1].value;
    const byValue = choices.find((c) => c.value === a);
    if (byValue) return byValue.value;
    console.log(yellow('invalid choice'));
  }
  return choices[choices.length - 1].value;
}

function needPython() {
  const py = findPython();
  if (!py) {
    console.error(red('Python >= 3.9 not found (set GPU_WORKER_PYTHON to its path)'));
    process.exit(1);
  }
  return py;
}

// returns the python to run cli.py with, creating / filling the venv on first use
async function ensureSetup(opts, allowPrompt) {
  if (opts.useSystemPython) {
    const py = needPython();
    console.log(green(`using system Python: ${py}`));
    return py;
  }
  const existing = venvPython();
  if (existing) return existing;
  let skipInstall = opts.skipInstall;
  if (allowPrompt) {
    const mode = await choose('No virtual environment found. How should the worker run?', [
      { name: 'create a virtual environment and install dependencies (recommended)', value: 'venv' },
      { name: 'create a virtual environment, skip dependency installation', value: 'venv-skip' },
      { name: 'use the system Python as is', value: 'system' },
    ]);
    if (mode === 'system') return ensureSetup(Object.assign({}, opts, { useSystemPython: true }), false);
    if (mode === 'venv-skip') skipInstall = true;
  }
  const py = needPython();
  console.log(cyan('first run: setting up the worker environment'));
  const reuse = torchKind(py) === 'hip';
  if (!createVenv(py, reuse)) process.exit(1);
  const vpy = venvPython() || (DRY ? py : null);
  if (!vpy) process.exit(1);
  if (!skipInstall && !installDependencies(vpy)) process.exit(1);
  return vpy;
}

function runCli(py, args) {
  closeInput();            // the wizard child reads the terminal itself
  const cli = path.join(PKG_DIR, 'cli.py');
  if (DRY) {
    console.log(`[dry-run] ${py} ${cli} ${args.join(' ')}`);
    process.exit(0);
  }
  const child = spawn(py, [cli].concat(args), { stdio: 'inherit', cwd: process.cwd() });
  const fwd = (sig) => () => child.kill(sig);
  process.on('SIGINT', fwd('SIGINT'));
  process.on('SIGTERM', fwd('SIGTERM'));
  child.on('error', (e) => { console.error(red(`failed to start Python: ${e.message}`)); process.exit(1); });
  child.on('exit', (code, signal) => process.exit(code === null ? (signal ? 1 : 0) : code));
}

// ------------------------------------------------------------------ CLI
const HELP = `gpu-worker ${VERSION} — distributed inference worker (AMD Instinct MI355X)

usage: gpu-worker [options] [command] [args]

commands:
  (none)              interactive menu (first run: environment setup)
  setup               create .venv and install dependencies
  install             (re)install dependencies into .venv and build the HIP kernels
  configure           configuration wizard
  start [-c FILE]     start the worker (runs the wizard if FILE does not exist; default config.yaml)
  status              registration / server status
  set KEY VALUE       set a config value (dotted key)
  check               probe GPUs, ROCm and dependencies
  bench               local engine throughput check

options:
  --use-system-python   run with the system Python (no venv, no installs)
  --skip-install        create the venv but do not install dependencies
  -h, --help            this help
  -V, --version         version

environment:
  GPU_WORKER_PYTHON       Python interpreter to use
  GPU_WORKER_WHEELHOUSE   install offline from this wheel directory
  GPU_WORKER_ROCM_VERSION override the detected ROCm release (torch wheel index)
`;

function parseArgs(argv) {
  const opts = { useSystemPython: false, skipInstall: false, help: false, version: false, config: 'config.yaml' };
  const rest = [];
  for (let i = 0; i < argv.length; i++) {
    const a = argv[i];
    if (a === '--use-system-python') opts.useSystemPython = true;
    else if (a === '--skip-install') opts.skipInstall = true;
    else if (a === '-h' || a === '--help') opts.help = true;
    else if (a === '-V' || a === '--version') opts.version = true;
    else if ((a === '-c' || a === '--config') && i + 1 < argv.length) opts.config = argv[++i];
    else if (a.startsWith('--config=')) opts.config = a.slice(9);
    else rest.push(a);
  }
  return { opts, command: rest[0] || 'quick', args: rest.slice(1) };
}

async function main() {
  const { opts, command, args } = parseArgs(process.argv.slice(2));
  if (opts.version) { console.log(VERSION); return; }
  if (opts.help || command === 'help') { console.log(HELP); return; }
  switch (command) {
    case 'setup': {
      if (opts.useSystemPython) { console.log(yellow('setup only manages the virtual environment')); return; }
      const py = needPython();
      if (!venvPython() && !createVenv(py, torchKind(py) === 'hip')) process.exit(1);
      if (!opts.skipInstall && !installDependencies(venvPython() || py)) process.exit(1);
      console.log(green('\nsetup complete. next: gpu-worker configure, then gpu-worker start'));
      return;
    }
    case 'install': {
      if (opts.useSystemPython) {
        runCli(needPython(), ['install']);        // deps check + kernel build in the system env
        return;
      }
      const py = await ensureSetup(Object.assign({}, opts, { skipInstall: true }), false);
      if (!installDependencies(py)) process.exit(1);
      return;
    }
    case 'start': {
      const py = await ensureSetup(opts, false);
      const cfg = path.resolve(opts.config);
      if (!fs.existsSync(cfg)) {
        console.log(yellow(`no config file at ${cfg} — starting the configuration wizard`));
        runCli(py, ['--config', cfg, 'configure']);
        return;
      }
      runCli(py, ['--config', cfg, 'start'].concat(args));
      return;
    }
    case 'configure': case 'status': case 'check': case 'bench':
      runCli(await ensureSetup(opts, false), ['--config', path.resolve(opts.config), command].concat(args));
      return;
    case 'set':
      if (args.length !== 2) { console.error(red('usage: gpu-worker set KEY VALUE')); process.exit(2); }
      runCli(await ensureSetup(opts, false), ['--config', path.resolve(opts.config), 'set'].concat(args));
      return;
    case 'quick': {
      const py = await ensureSetup(opts, true);
      console.log(cyan(bold('\n  GPU Worker — distributed inference node (MI355X)\n')));
      const action = await choose('What do you want to do?', [
        { name: 'start the worker', value: 'start' },
        { name: 'configuration wizard', value: 'configure' },
        { name: 'status', value: 'status' },
        { name: 'check GPUs / ROCm / dependencies', value: 'check' },
        { name: 'install dependencies / build kernels', value: 'install' },
        { name: 'exit', value: 'exit' },
      ]);
      if (action === 'exit') process.exit(0);
      if (action === 'install' && !opts.useSystemPython) { if (!installDependencies(py)) process.exit(1); return; }
      if (action === 'start' && !fs.existsSync(path.resolve(opts.config))) {
        console.log(yellow('\nno config file yet — configuring first\n'));
        runCli(py, ['--config', path.resolve(opts.config), 'configure']);
        return;
      }
      runCli(py, ['--config', path.resolve(opts.config), action]);
      return;
    }
    default:
      console.error(red(`unknown command: ${command}`));
      console.log(HELP);
      process.exit(2);
  }
}

module.exports = { parseArgs, rocmVersion, torchIndexUrl, filterRequirements, planInstall };

if (require.main === module) {
  main().catch((e) => { console.error(red(e && e.stack ? e.stack : String(e))); process.exit(1); });
}
