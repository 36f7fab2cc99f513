"""Initial schema: workers, jobs, enterprises, API keys, usage, bills, price plans, worker summaries.

The reference shipped no ORM or revisions (its models were git-ignored,
SURVEY Appendix D); this revision materialises the reconstructed schema
from ``app.models`` so SQLite and Postgres deployments start identical.

Revision ID: 0001_initial
Revises:
"""
from alembic import op

from app.db.database import Base
from app.models import models, usage  # noqa: F401

revision = "0001_initial"
down_revision = None
branch_labels = None
depends_on = None


def upgrade() -> None:
    Base.metadata.create_all(bind=op.get_bind())


def downgrade() -> None:
    Base.metadata.drop_all(bind=op.get_bind())
