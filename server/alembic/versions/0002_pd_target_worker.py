"""P/D job path: ``jobs.target_worker_id`` (decode phase pinned to the chosen worker).

Revision ID: 0002_pd_target_worker
Revises: 0001_initial
"""
import sqlalchemy as sa
from alembic import op

revision = "0002_pd_target_worker"
down_revision = "0001_initial"
branch_labels = None
depends_on = None


def upgrade() -> None:
    cols = {c["name"] for c in sa.inspect(op.get_bind()).get_columns("jobs")}
    if "target_worker_id" not in cols:      # 0001 on a newer model already created it
        op.add_column("jobs", sa.Column("target_worker_id", sa.String(36), nullable=True))
        op.create_index("ix_jobs_target_worker_id", "jobs", ["target_worker_id"])


def downgrade() -> None:
    op.drop_index("ix_jobs_target_worker_id", table_name="jobs")
    op.drop_column("jobs", "target_worker_id")
