"""Control plane: FastAPI job/worker/admin API over SQLAlchemy (SQLite or Postgres)."""
