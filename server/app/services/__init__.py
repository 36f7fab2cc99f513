"""Control-plane services (scheduling, P/D, reliability, task guarantee, security,
worker config, geo, usage/billing, privacy, observability)."""
