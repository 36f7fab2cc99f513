#!/bin/bash
# Deploy the control plane (and optionally a local MI355X worker) with docker compose.
#   scripts/deploy.sh server        # postgres + redis + API server
#   scripts/deploy.sh worker        # + local GPU worker (needs /dev/kfd, /dev/dri)
set -euo pipefail
cd "$(dirname "$0")/.."
mode=${1:-server}
command -v docker >/dev/null || { echo "docker is required"; exit 1; }
compose="docker compose"; $compose version >/dev/null 2>&1 || compose="docker-compose"
[ -f .env ] || { echo "no .env: using defaults from .env.example"; cp .env.example .env; }
case $mode in
  server) $compose up -d --build postgres redis server ;;
  worker)
    [ -e /dev/kfd ] || { echo "no /dev/kfd: this host has no ROCm GPU"; exit 1; }
    $compose --profile with-worker up -d --build ;;
  *) echo "usage: $0 [server|worker]"; exit 2 ;;
esac
port=$(grep -E '^SERVER_PORT=' .env | cut -d= -f2); port=${port:-8000}
for i in $(seq 1 30); do
  if curl -fs "http://localhost:$port/health" >/dev/null; then echo "server healthy on :$port"; exit 0; fi
  sleep 2
done
echo "server did not become healthy"; $compose logs --tail=50 server; exit 1
