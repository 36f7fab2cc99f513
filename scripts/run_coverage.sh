#!/bin/bash
# CPU test suite under coverage (needs the `coverage` package; not in the offline image).
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "import coverage" 2>/dev/null || { echo "coverage is not installed: pip install coverage"; exit 1; }
mkdir -p manual_tmp/coverage
data="manual_tmp/coverage/.coverage.$(date +%Y%m%d%H%M%S).$$"
python -m coverage run --source=dgi,worker,server/app,common,sdk --data-file "$data" -m pytest -q -m "not gpu"
python -m coverage report --data-file "$data" --fail-under "${FAIL_UNDER:-70}"
