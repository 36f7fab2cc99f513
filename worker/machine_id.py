"""Stable machine fingerprint (reference worker/machine_id.py:17-200).

Hash of OS/platform identity, MAC, the OS machine-id and the GPU inventory.
GPU identity comes from torch plus ``amd-smi`` / ``rocm-smi`` unique ids on
ROCm (the reference queried ``nvidia-smi``).  Persisted as JSON and reused
while the hardware hash is unchanged.
"""
from __future__ import annotations

import hashlib
import json
import os
import platform
import subprocess  # module-level so callers/tests can patch machine_id.subprocess
import uuid
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, Optional


class MachineFingerprint:
    FINGERPRINT_FILE = ".gpu_worker_fingerprint"

    @classmethod
    def generate(cls) -> Dict[str, Any]:
        data: Dict[str, Any] = {
            "platform": platform.system(), "platform_release": platform.release(),
            "platform_version": platform.version(), "architecture": platform.machine(),
            "processor": platform.processor(), "hostname": platform.node(),
            "mac_address": cls._get_mac_address(), "machine_id": cls._get_machine_id(),
        }
        gpu = cls._get_gpu_info()
        if gpu:
            data["gpu"] = gpu
        digest = hashlib.sha256(json.dumps(data, sort_keys=True).encode()).hexdigest()
        return {"machine_id": digest[:32], "hardware_hash": digest, "details": data,
                "generated_at": cls._get_timestamp()}

    @classmethod
    def _get_mac_address(cls) -> str:
        try:
            mac = f"{uuid.getnode():012X}"
            return ":".join(mac[i:i + 2] for i in range(0, 12, 2))
        except Exception:
            return "unknown"

    @classmethod
    def _run(cls, args) -> Optional[str]:
        try:
            r = subprocess.run(args, capture_output=True, text=True, timeout=10)
        except Exception:
            return None
        return r.stdout if getattr(r, "returncode", 1) == 0 else None

    @classmethod
    def _get_machine_id(cls) -> str:
        for p in ("/etc/machine-id", "/var/lib/dbus/machine-id"):
            if os.path.exists(p):
                try:
                    v = Path(p).read_text().strip()
                    if v:
                        return v
                except OSError:
                    pass
        system = platform.system()
        if system == "Darwin":
            out = cls._run(["ioreg", "-rd1", "-c", "IOPlatformExpertDevice"]) or ""
            for line in out.splitlines():
                if "IOPlatformUUID" in line:
                    return line.split('"')[-2]
        if system == "Windows":
            out = cls._run(["wmic", "csproduct", "get", "UUID"]) or ""
            rows = [r.strip() for r in out.strip().splitlines() if r.strip()]
            if len(rows) > 1:
                return rows[1]
        return str(uuid.getnode())

    @classmethod
    def _get_gpu_info(cls) -> Optional[Dict[str, Any]]:
        try:
            import torch
            n = torch.cuda.device_count()
            if n == 0:
                return None
            name = torch.cuda.get_device_properties(0).name
        except Exception:
            return None
        return {"count": n, "name": name, "uuid": cls._get_gpu_uuid()}

    @classmethod
    def _get_gpu_uuid(cls) -> Optional[str]:
        out = cls._run(["amd-smi", "static", "--asic", "--json"])
        if out:
            try:
                js = json.loads(out)
                items = js if isinstance(js, list) else [js]
                for it in items:
                    asic = it.get("asic", {}) if isinstance(it, dict) else {}
                    for key in ("asic_serial", "device_id"):
                        if asic.get(key):
                            return str(asic[key])
            except ValueError:
                pass
        out = cls._run(["rocm-smi", "--showuniqueid"])
        if out:
            for line in out.splitlines():
                if "Unique ID" in line:
                    return line.split(":")[-1].strip()
        return None

    @classmethod
    def _get_timestamp(cls) -> str:
        return datetime.utcnow().isoformat() + "Z"

    @classmethod
    def get_or_create(cls, storage_path: Optional[str] = None) -> Dict[str, Any]:
        path = Path(storage_path or Path.home() / cls.FINGERPRINT_FILE)
        current = cls.generate()
        if path.is_file():
            try:
                saved = json.loads(path.read_text(encoding="utf-8"))
                if saved.get("hardware_hash") == current["hardware_hash"] and saved.get("machine_id"):
                    return saved
            except (OSError, ValueError):
                pass
        try:
            path.parent.mkdir(parents=True, exist_ok=True)
            path.write_text(json.dumps(current, indent=2), encoding="utf-8")
        except OSError:
            pass
        return current

    @classmethod
    def get_machine_id(cls) -> str:
        return cls.get_or_create()["machine_id"]


def get_machine_id() -> str:
    return MachineFingerprint.get_machine_id()


def get_full_fingerprint() -> Dict[str, Any]:
    return MachineFingerprint.get_or_create()
