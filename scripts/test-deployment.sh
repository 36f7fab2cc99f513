#!/bin/bash
# Smoke-test a running deployment: health, regions, queue stats, one sync LLM job.
set -euo pipefail
URL=${1:-http://localhost:8000}
echo "health:  $(curl -fs $URL/health)"
echo "regions: $(curl -fs $URL/regions | head -c 200)"
echo "queue:   $(curl -fs $URL/api/v1/jobs/stats/queue)"
echo "workers: $(curl -fs $URL/api/v1/workers | head -c 300)"
body='{"type":"llm","params":{"messages":[{"role":"user","content":"hello"}],"max_tokens":16,"temperature":0}}'
code=$(curl -s -o /tmp/dgi_job.json -w '%{http_code}' -X POST "$URL/api/v1/jobs/sync?timeout=120&wait_for_worker=false" \
  -H 'Content-Type: application/json' -d "$body")
echo "sync job HTTP $code: $(head -c 400 /tmp/dgi_job.json)"
[ "$code" = 200 ] || [ "$code" = 503 ]
