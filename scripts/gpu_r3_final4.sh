#!/bin/bash
# Final check of the tree: full GPU suite + smoke first, then 8B decode TPOT + kernel table.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
bash scripts/gpu_r3_suite.sh || exit 1
bash scripts/gpu_r3_decode_prof.sh || exit 1
rm -rf gpurun_out/prof_dec8b
