"""npm launcher (worker/bin/gpu-worker.js): setup flow, menu and forwarding.

The reference's launcher (worker/bin/gpu-worker.js:187-433) creates a venv on
first run, installs torch + requirements, offers an interactive menu and
forwards commands to cli.py.  These tests run ours in dry-run mode
(GPU_WORKER_DRY_RUN=1: commands are printed, nothing is created or installed)
with piped menu answers.
"""
import json
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
JS = ROOT / "worker" / "bin" / "gpu-worker.js"
pytestmark = pytest.mark.skipif(shutil.which("node") is None, reason="node not installed")


def _run(args, stdin="", **env):
    e = dict(os.environ, GPU_WORKER_DRY_RUN="1", GPU_WORKER_PYTHON="python3", **env)
    r = subprocess.run(["node", str(JS)] + args, input=stdin, capture_output=True, text=True, env=e,
                       cwd=str(ROOT / "worker"), timeout=120)
    return r.returncode, r.stdout + r.stderr


def _node(expr):
    r = subprocess.run(["node", "-e", f"const m=require({json.dumps(str(JS))}); console.log(JSON.stringify({expr}))"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


def test_syntax_help_version():
    assert subprocess.run(["node", "--check", str(JS)]).returncode == 0
    rc, out = _run(["--version"])
    assert rc == 0 and out.strip() == json.loads((ROOT / "worker/package.json").read_text())["version"]
    rc, out = _run(["--help"])
    assert rc == 0 and all(c in out for c in ("setup", "install", "configure", "start", "status", "set KEY VALUE"))
    rc, out = _run(["frobnicate"])
    assert rc == 2 and "unknown command" in out


def test_rocm_wheel_index_and_requirements_filter():
    assert _node("m.torchIndexUrl('7.2')") == "https://download.pytorch.org/whl/rocm7.0"
    assert _node("m.torchIndexUrl('6.3')") == "https://download.pytorch.org/whl/rocm6.3"
    assert _node("m.torchIndexUrl('5.7')") is None and _node("m.torchIndexUrl(null)") is None
    assert _node("m.rocmVersion({GPU_WORKER_ROCM_VERSION: '6.4'})") == "6.4"
    assert _node("m.filterRequirements('torch>=2.0\\nhttpx>=0.25\\n# c\\ntorchvision\\ntorch')") == \
        "httpx>=0.25\n# c\ntorchvision"
    # torch already a ROCm build: only the requirements are installed
    plan = _node("m.planInstall('py', {GPU_WORKER_TORCH_KIND: 'hip'})")
    assert plan["torch"] == "hip" and len(plan["steps"]) == 1 and "-r" in plan["steps"][0]
    # no torch: the ROCm wheel index of the installed release
    plan = _node("m.planInstall('py', {GPU_WORKER_TORCH_KIND: '', GPU_WORKER_ROCM_VERSION: '6.4'})")
    assert plan["steps"][0][-2:] == ["--index-url", "https://download.pytorch.org/whl/rocm6.4"]
    # offline wheelhouse: --no-index everywhere
    plan = _node("m.planInstall('py', {GPU_WORKER_TORCH_KIND: 'cpu', GPU_WORKER_WHEELHOUSE: '/w'})")
    assert all("--no-index" in s and "/w" in s for s in plan["steps"])
    assert _node("m.parseArgs(['--skip-install', 'start', '-c', 'a.yaml']).opts") == {
        "useSystemPython": False, "skipInstall": True, "help": False, "version": False, "config": "a.yaml"}


@pytest.mark.skipif((ROOT / "worker" / ".venv").exists(), reason="a real venv exists")
def test_first_run_menu_creates_venv_then_forwards():
    # answer 1 = create venv + install, then 3 = status
    rc, out = _run([], stdin="1\n3\n", GPU_WORKER_TORCH_KIND="")
    assert rc == 0, out
    assert "-m venv" in out and "pip install" in out and "cli.py install" in out
    assert out.rstrip().endswith("status")
    # "use the system Python" skips the venv entirely; 6 = exit
    rc, out = _run([], stdin="3\n6\n")
    assert rc == 0 and "-m venv" not in out and "using system Python" in out


def test_start_without_config_runs_wizard_and_forwards_commands(tmp_path):
    cfg = tmp_path / "c.yaml"
    rc, out = _run(["--use-system-python", "start", "-c", str(cfg)])
    assert rc == 0 and f"--config {cfg} configure" in out
    cfg.write_text("server: {url: http://127.0.0.1:8000}\n")
    rc, out = _run(["--use-system-python", "start", "-c", str(cfg)])
    assert rc == 0 and f"--config {cfg} start" in out
    rc, out = _run(["--use-system-python", "set", "engine.type", "native"])
    assert rc == 0 and out.rstrip().endswith("set engine.type native")
    rc, out = _run(["--use-system-python", "set", "only-key"])
    assert rc == 2
