"""Server settings (env / ``.env``; same field and variable names as the reference's
server/app/config.py:7-51).  Implemented on plain pydantic so it does not need
``pydantic-settings``."""
from __future__ import annotations

import os
from typing import Any, Dict

from pydantic import BaseModel, field_validator


def _read_dotenv(path: str = ".env") -> Dict[str, str]:
    out: Dict[str, str] = {}
    if not os.path.exists(path):
        return out
    for line in open(path, encoding="utf-8"):
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        out[k.strip()] = v.strip().strip('"').strip("'")
    return out


class Settings(BaseModel):
    app_name: str = "Distributed GPU Inference"
    debug: bool = False
    region: str = "asia-east"
    database_url: str = "sqlite:///./inference.db"
    redis_url: str = "redis://localhost:6379/0"
    secret_key: str = "change-me-in-production"
    api_key_header: str = "X-API-Key"
    worker_token_header: str = "X-Worker-Token"
    heartbeat_timeout_seconds: int = 90
    job_timeout_seconds: int = 300
    stale_job_check_interval: int = 30
    rate_limit_per_minute: int = 60
    enable_cross_region: bool = True
    cross_region_penalty: float = 0.3
    require_signature: bool = False
    admin_token: str = ""           # empty = admin API open (reference behaviour); set to require X-Admin-Token
    geo_lookup_enabled: bool = False  # network GeoIP lookups are opt-in (offline by default)

    @field_validator("debug", "enable_cross_region", "require_signature", "geo_lookup_enabled", mode="before")
    @classmethod
    def _boolish(cls, v: Any) -> bool:
        if isinstance(v, str):
            return v.strip().lower() in ("1", "true", "yes", "on")
        return bool(v)

    @classmethod
    def from_env(cls) -> "Settings":
        env = {**_read_dotenv(), **os.environ}
        data = {}
        for name in cls.model_fields:
            for key in (name.upper(), name):
                if key in env:
                    data[name] = env[key]
                    break
        return cls(**data)


settings = Settings.from_env()
