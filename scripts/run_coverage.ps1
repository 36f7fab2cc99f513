# CPU test suite under coverage (PowerShell twin of scripts/run_coverage.sh).
$ErrorActionPreference = "Stop"
Set-Location (Join-Path (Split-Path -Parent $MyInvocation.MyCommand.Path) "..")
New-Item -ItemType Directory -Force "manual_tmp/coverage" | Out-Null
$data = "manual_tmp/coverage/.coverage.$(Get-Date -Format yyyyMMddHHmmss).$PID"
$fail = if ($env:FAIL_UNDER) { $env:FAIL_UNDER } else { 70 }
python -m coverage run --source=dgi,worker,server/app,common,sdk --data-file $data -m pytest -q -m "not gpu"
python -m coverage report --data-file $data --fail-under $fail
