#!/usr/bin/env python3
"""2-rank shared-GPU check of the RCCL transport log (dgi.parallel.fabric.rccl_transports):
set up a 1P+1D layout, warm the pairs, and print what the rank's RCCL INIT log shows right after
set-up and again at the end (is the file flushed while the process runs?)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgi.parallel.fabric import Fabric, rccl_transports, rccl_log_path  # noqa: E402
from dgi.parallel.plan import NodeLayout  # noqa: E402

f = Fabric()
lay = NodeLayout("pd", [0], [1])
f.setup_layout(lay)
after_setup = rccl_transports()
f.barrier()
path = os.environ.get("NCCL_DEBUG_FILE") or rccl_log_path()
size = os.path.getsize(path) if os.path.exists(path) else None
print(json.dumps({"rank": f.rank, "path": path, "exists": os.path.exists(path), "size": size,
                  "env": {k: os.environ.get(k) for k in ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE")},
                  "after_setup": after_setup}), flush=True)
if f.rank == 0 and os.path.exists(path):
    with open(path, errors="replace") as fh:
        lines = fh.readlines()
    print(json.dumps({"lines": len(lines), "head": lines[:5], "via": [x for x in lines if "via" in x][:8]}), flush=True)
f.close()
