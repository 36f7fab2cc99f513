"""Worker CLI (reference worker/cli.py:653-873): `set` writes dotted keys, `start -c` is accepted
after the subcommand (reference bug E-27)."""
import importlib.util
import os

import yaml

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli():
    spec = importlib.util.spec_from_file_location("dgi_worker_cli", os.path.join(_ROOT, "worker", "cli.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_set_writes_nested_key(tmp_path, capsys):
    cli = _cli()
    cfg = tmp_path / "c.yaml"
    assert cli.main(["--config", str(cfg), "set", "load_control.max_concurrent_jobs", "128"]) == 0
    assert cli.main(["--config", str(cfg), "set", "gpu.layout", "pdpp"]) == 0
    data = yaml.safe_load(cfg.read_text())
    assert data["load_control"]["max_concurrent_jobs"] == 128
    assert data["gpu"]["layout"] == "pdpp"


def test_start_accepts_config_after_subcommand(monkeypatch, tmp_path):
    cli = _cli()
    seen = {}
    monkeypatch.setattr(cli, "cmd_start", lambda a: seen.setdefault("config", a.config) and 0)

    # the parser binds fn at construction, so re-dispatch through argparse with the patched function
    import argparse
    real = argparse.ArgumentParser.parse_args

    def parse(self, args=None, namespace=None):
        ns = real(self, args, namespace)
        if getattr(ns, "cmd", None) == "start":
            ns.fn = cli.cmd_start
        return ns
    monkeypatch.setattr(argparse.ArgumentParser, "parse_args", parse)
    cli.main(["start", "-c", str(tmp_path / "x.yaml")])
    assert seen["config"] == str(tmp_path / "x.yaml")
