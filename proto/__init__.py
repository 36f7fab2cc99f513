"""Wire contract of the worker data plane (``inference.proto``, unchanged from the reference)."""
