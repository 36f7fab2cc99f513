"""Shared observability for the worker process.

The metric names / labels, tracing manager and route factory live in the
control plane's ``server/app/services/observability.py`` (reference
observability.py:20-488).  The worker loads that file by path so it does not
pull in the server package's settings or database.
"""
from __future__ import annotations

import os
import sys


def load_observability():
    """The control plane's observability module (metrics names, tracing), loaded
    by path so the worker does not need the server package's settings."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "server", "app", "services",
                        "observability.py")
    if "dgi_observability" in sys.modules:
        return sys.modules["dgi_observability"]
    spec = importlib.util.spec_from_file_location("dgi_observability", path)
    if spec is None or not os.path.exists(path):
        return None
    mod = importlib.util.module_from_spec(spec)
    sys.modules["dgi_observability"] = mod
    spec.loader.exec_module(mod)
    return mod
