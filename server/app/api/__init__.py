"""HTTP routers (jobs, workers, admin) — route surface of reference server/app/api/*.py."""
