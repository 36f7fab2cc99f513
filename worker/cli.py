"""``gpu-worker`` command line (reference worker/cli.py:72-877).

Commands: ``check`` (GPU / ROCm / dependency probe), ``configure``
(interactive wizard or flags → config.yaml), ``start``, ``status``
(credentials, server reachability, local engines), ``set KEY VALUE``
(dotted keys into config.yaml), ``bench`` (quick local engine throughput).
The reference's ``install`` downloaded CUDA wheels; on this platform the
ROCm PyTorch build is a prerequisite, so ``install`` only verifies it.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
from typing import Any, Dict, List, Optional

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import yaml  # noqa: E402

CONFIG_FILE = "config.yaml"
REGIONS = ["asia-east", "asia-south", "europe-west", "europe-east", "america-north", "america-south", "oceania"]
TASK_TYPES = ["llm", "image_gen", "vision", "whisper", "embedding"]
REQUIRED = ["torch", "httpx", "yaml", "pydantic", "fastapi", "uvicorn"]
OPTIONAL = ["transformers", "diffusers", "safetensors", "grpc"]


def _probe_rocm() -> Optional[Dict[str, Any]]:
    """GPU inventory via amd-smi (JSON) or rocm-smi, without initialising HIP in this process."""
    for cmd in (["amd-smi", "static", "--asic", "--vram", "--json"], ["rocm-smi", "--showproductname", "--json"]):
        if shutil.which(cmd[0]) is None:
            continue
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=20)
        except Exception:
            continue
        if r.returncode == 0 and r.stdout.strip():
            try:
                return {"tool": cmd[0], "data": json.loads(r.stdout)}
            except ValueError:
                return {"tool": cmd[0], "raw": r.stdout[:2000]}
    return None


def check_gpu() -> Dict[str, Any]:
    out: Dict[str, Any] = {"rocm": os.path.isdir("/opt/rocm"), "smi": _probe_rocm()}
    try:
        import torch
        out["torch"] = torch.__version__
        out["hip"] = getattr(torch.version, "hip", None)
        out["device_count"] = torch.cuda.device_count()
    except Exception as e:
        out["torch_error"] = str(e)
    try:
        from dgi import ops
        out["dgi_native_built"] = ops.native_available()
    except Exception as e:
        out["dgi_error"] = str(e)
    return out


def check_dependencies() -> Dict[str, bool]:
    import importlib.util
    return {m: importlib.util.find_spec(m) is not None for m in REQUIRED + OPTIONAL}


def load_yaml(path: str = CONFIG_FILE) -> Dict[str, Any]:
    if not os.path.exists(path):
        return {}
    with open(path, encoding="utf-8") as f:
        return yaml.safe_load(f) or {}


def save_yaml(data: Dict[str, Any], path: str = CONFIG_FILE) -> None:
    with open(path, "w", encoding="utf-8") as f:
        yaml.safe_dump(data, f, default_flow_style=False, allow_unicode=True, sort_keys=False)


def _coerce(v: str) -> Any:
    low = v.strip().lower()
    if low in ("true", "false"):
        return low == "true"
    if low in ("null", "none"):
        return None
    for cast in (int, float):
        try:
            return cast(v)
        except ValueError:
            pass
    if "," in v:
        return [x.strip() for x in v.split(",") if x.strip()]
    return v


def set_key(data: Dict[str, Any], dotted: str, value: Any) -> Dict[str, Any]:
    cur = data
    parts = dotted.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
        if not isinstance(cur, dict):
            raise ValueError(f"{p} is not a section")
    cur[parts[-1]] = value
    return data


def _ask(prompt: str, default: Any = None, choices: Optional[List[str]] = None) -> str:
    hint = f" [{default}]" if default is not None else ""
    if choices:
        prompt = f"{prompt} ({'/'.join(choices)})"
    while True:
        v = input(f"{prompt}{hint}: ").strip()
        if not v and default is not None:
            return str(default)
        if not choices or v in choices:
            return v


def wizard(existing: Dict[str, Any]) -> Dict[str, Any]:
    d = dict(existing)
    d.setdefault("server", {})["url"] = _ask("Control-plane URL", d.get("server", {}).get("url", "http://localhost:8000"))
    d["region"] = _ask("Region", d.get("region", "asia-east"), REGIONS)
    d["name"] = _ask("Worker name", d.get("name") or os.uname().nodename)
    types = _ask("Task types (comma separated)", ",".join(d.get("supported_types", ["llm"])))
    d["supported_types"] = [t.strip() for t in types.split(",") if t.strip() in TASK_TYPES]
    if "llm" in d["supported_types"]:
        llm = d.setdefault("engines", {}).setdefault("llm", {})
        llm["model_id"] = _ask("LLM model (preset or local path)", llm.get("model_id", "llama3-8b"))
        llm["backend"] = _ask("LLM backend", llm.get("backend", "mi355x"), ["mi355x", "native", "sglang", "vllm"])
    g = d.setdefault("gpu", {})
    ids = _ask("GPU ids for this worker (comma separated)", ",".join(map(str, g.get("device_ids", [0]))))
    g["device_ids"] = [int(x) for x in ids.split(",") if x.strip()]
    if len(g["device_ids"]) > 1:
        g["layout"] = _ask("Multi-GPU layout", g.get("layout", "pdpp"), ["pdpp", "pd", "pp"])
    lc = d.setdefault("load_control", {})
    lc["max_concurrent_jobs"] = int(_ask("Max concurrent jobs", lc.get("max_concurrent_jobs", 64)))
    lc["acceptance_rate"] = float(_ask("Acceptance rate 0-1", lc.get("acceptance_rate", 1.0)))
    dr = d.setdefault("direct", {})
    dr["enabled"] = _ask("Enable direct connections", "yes" if dr.get("enabled") else "no", ["yes", "no"]) == "yes"
    if dr["enabled"]:
        dr["port"] = int(_ask("Direct port", dr.get("port", 8080)))
        dr["public_url"] = _ask("Public URL", dr.get("public_url") or f"http://{d['name']}:{dr['port']}")
    return d


def cmd_check(a) -> int:
    print(json.dumps({"gpu": check_gpu(), "dependencies": check_dependencies()}, indent=2, default=str))
    return 0


def cmd_install(a) -> int:
    deps = check_dependencies()
    missing = [m for m in REQUIRED if not deps[m]]
    if missing:
        print("missing required packages:", ", ".join(missing))
        print("install a ROCm PyTorch build plus: pip install httpx pyyaml pydantic fastapi uvicorn")
        return 1
    print("all required packages present")
    try:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from dgi.build import build
        build()
        print("dgi HIP kernels built for gfx950")
    except Exception as e:
        print("dgi kernels not built:", e)
    return 0


def cmd_configure(a) -> int:
    data = load_yaml(a.config)
    if a.non_interactive:
        for kv in a.set or []:
            k, v = kv.split("=", 1)
            set_key(data, k, _coerce(v))
    else:
        data = wizard(data)
    save_yaml(data, a.config)
    print(f"wrote {a.config}")
    return 0


def cmd_set(a) -> int:
    data = set_key(load_yaml(a.config), a.key, _coerce(a.value))
    save_yaml(data, a.config)
    print(f"{a.key} = {data_get(data, a.key)!r}")
    return 0


def data_get(d: Dict[str, Any], dotted: str) -> Any:
    for p in dotted.split("."):
        d = d.get(p) if isinstance(d, dict) else None
    return d


def cmd_status(a) -> int:
    from config import load_config
    cfg = load_config(a.config)
    info: Dict[str, Any] = {"worker_id": cfg.worker_id, "server": cfg.server.url, "region": cfg.region,
                            "supported_types": cfg.supported_types, "registered": bool(cfg.token)}
    try:
        import httpx
        r = httpx.get(f"{cfg.server.url.rstrip('/')}/health", timeout=5)
        info["server_health"] = r.json()
        if cfg.worker_id and cfg.token:
            from api_client import APIClient
            info["credentials_valid"] = APIClient(cfg.server.url).verify_credentials(cfg.worker_id, cfg.token)
    except Exception as e:
        info["server_error"] = str(e)
    print(json.dumps(info, indent=2, default=str))
    return 0


def cmd_start(a) -> int:
    import logging
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    from main import Worker
    Worker(config_path=a.config).start()
    return 0


def cmd_bench(a) -> int:
    """Quick local throughput check of the configured LLM engine (no control plane)."""
    import time
    from config import load_config
    from engines import create_llm_engine
    cfg = load_config(a.config)
    ecfg = cfg.engine_config("llm")
    if a.model:
        ecfg["model_id"] = a.model
    eng = create_llm_engine(ecfg)
    eng.load_model()
    params = [{"messages": [{"role": "user", "content": f"request {i} " + "x" * a.prompt_chars}],
               "max_tokens": a.max_tokens, "temperature": 0.0} for i in range(a.requests)]
    t0 = time.time()
    outs = eng.batch_inference(params)
    dt = time.time() - t0
    toks = sum(o["usage"]["completion_tokens"] for o in outs)
    print(json.dumps({"requests": a.requests, "completion_tokens": toks, "seconds": round(dt, 3),
                      "tokens_per_second": round(toks / dt, 1)}))
    eng.unload_model()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="gpu-worker", description="Distributed GPU inference worker")
    ap.add_argument("--config", default=CONFIG_FILE)
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("check", help="probe GPU, ROCm and dependencies").set_defaults(fn=cmd_check)
    sub.add_parser("install", help="verify dependencies and build the HIP kernels").set_defaults(fn=cmd_install)
    c = sub.add_parser("configure", help="interactive configuration wizard")
    c.add_argument("--non-interactive", action="store_true")
    c.add_argument("--set", action="append", metavar="KEY=VALUE")
    c.set_defaults(fn=cmd_configure)
    st = sub.add_parser("start", help="start the worker")
    # reference bug E-27: `gpu-worker start -c config.yaml` was rejected; accept it after the subcommand too
    st.add_argument("-c", "--config", dest="start_config", default=None)
    st.set_defaults(fn=cmd_start)
    sub.add_parser("status", help="show registration / server status").set_defaults(fn=cmd_status)
    s = sub.add_parser("set", help="set a config value (dotted key)")
    s.add_argument("key")
    s.add_argument("value")
    s.set_defaults(fn=cmd_set)
    b = sub.add_parser("bench", help="local engine throughput check")
    b.add_argument("--model", default=None)
    b.add_argument("--requests", type=int, default=32)
    b.add_argument("--max-tokens", type=int, default=64)
    b.add_argument("--prompt-chars", type=int, default=200)
    b.set_defaults(fn=cmd_bench)
    a = ap.parse_args(argv)
    if getattr(a, "start_config", None):
        a.config = a.start_config
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
