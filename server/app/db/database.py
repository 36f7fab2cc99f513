"""Database engine and sessions (reference server/app/db/database.py:7-28).

Synchronous SQLAlchemy 2.0 sessions; FastAPI runs DB-touching endpoints in its
thread pool, and async services use ``run_db`` to stay off the event loop.
Async driver URLs from the reference (``sqlite+aiosqlite``, ``postgresql+asyncpg``)
are mapped to their synchronous equivalents.
"""
from __future__ import annotations

from typing import Iterator

from sqlalchemy import create_engine
from sqlalchemy.orm import DeclarativeBase, Session, sessionmaker
from sqlalchemy.pool import StaticPool

from app.config import settings


def normalize_url(url: str) -> str:
    url = url.replace("sqlite+aiosqlite", "sqlite").replace("postgresql+asyncpg", "postgresql+psycopg")
    return url


def make_engine(url: str):
    url = normalize_url(url)
    if url.startswith("sqlite"):
        kw = {"connect_args": {"check_same_thread": False}}
        if ":memory:" in url or url in ("sqlite://", "sqlite:///"):
            kw["poolclass"] = StaticPool
        return create_engine(url, **kw)
    return create_engine(url, pool_pre_ping=True, pool_size=20, max_overflow=20)


class Base(DeclarativeBase):
    pass


engine = make_engine(settings.database_url)
SessionLocal = sessionmaker(bind=engine, expire_on_commit=False)
AsyncSessionLocal = SessionLocal  # name kept for callers of the reference API


def get_db() -> Iterator[Session]:
    db = SessionLocal()
    try:
        yield db
    finally:
        db.close()


def init_db() -> None:
    from app.models import models, usage  # noqa: F401  (register tables)
    Base.metadata.create_all(bind=engine)
