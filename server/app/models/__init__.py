"""ORM models reconstructed from the reference's usage sites;
the reference snapshot itself lacks ``server/app/models`` (excluded by .gitignore)."""
