"""Serving front-ends of the native runtime (node server)."""
