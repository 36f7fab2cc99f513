"""Node topology from the KFD sysfs tree: which GPUs share a direct xGMI link.

An 8x MI355X node is a full xGMI mesh: every GPU has one link (7 per GPU) to
each peer, so every prefill -> decode pair and every pipeline hop is one hop
and layouts need no placement search.  The runtime still checks it at start-up
(``bench.py`` reports ``extra.topology``) and ``order_stages`` keeps adjacent
pipeline stages on direct xGMI links when a node is not a full mesh (partial
partitions, PCIe-attached boards).

KFD layout: ``/sys/class/kfd/kfd/topology/nodes/<n>/gpu_id`` (0 on CPU nodes),
``nodes/<n>/properties`` (``simd_count``) and ``nodes/<n>/io_links/<m>/properties`` (``type``: 11 = xGMI,
2 = PCIe; ``node_to``; ``weight``: lower is closer; ``max_bandwidth``).
GPU nodes in node-id order are the HIP device ordinals.
"""
from __future__ import annotations

import itertools
import os
from typing import Optional

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
LINK_XGMI = 11
LINK_PCIE = 2


def _props(path: str) -> dict:
    out = {}
    try:
        with open(path) as f:
            for ln in f:
                k, _, v = ln.strip().partition(" ")
                if v.strip().lstrip("-").isdigit():
                    out[k] = int(v)
    except OSError:
        pass
    return out


def _is_gpu(node_dir: str) -> bool:
    """KFD exposes the GPU id in its own ``gpu_id`` file (0 on CPU nodes); the
    ``properties`` file has ``simd_count`` > 0 for GPUs."""
    try:
        with open(os.path.join(node_dir, "gpu_id")) as f:
            return int(f.read().strip() or 0) != 0
    except (OSError, ValueError):
        return _props(os.path.join(node_dir, "properties")).get("simd_count", 0) > 0


def read_topology(root: str = KFD_NODES) -> Optional[dict]:
    """{"gpus": n, "links": {(i, j): {"type", "weight", "max_bw"}}} over HIP ordinals,
    or None when the KFD tree is absent (CPU boxes)."""
    if not os.path.isdir(root):
        return None
    nodes = sorted(int(n) for n in os.listdir(root) if n.isdigit())
    gpu_nodes = [n for n in nodes if _is_gpu(os.path.join(root, str(n)))]
    ordinal = {n: i for i, n in enumerate(gpu_nodes)}
    links = {}
    for n in gpu_nodes:
        ldir = os.path.join(root, str(n), "io_links")
        if not os.path.isdir(ldir):
            continue
        for m in os.listdir(ldir):
            p = _props(os.path.join(ldir, m, "properties"))
            to = p.get("node_to")
            if to in ordinal:
                links[(ordinal[n], ordinal[to])] = {"type": p.get("type"), "weight": p.get("weight", 0),
                                                    "max_bw": p.get("max_bandwidth", 0)}
    return {"gpus": len(gpu_nodes), "links": links}


def summary(topo: Optional[dict]) -> Optional[dict]:
    """What the bench JSON reports: GPU count, xGMI link count, full-mesh flag."""
    if topo is None:
        return None
    n = topo["gpus"]
    xgmi = {k for k, v in topo["links"].items() if v["type"] == LINK_XGMI}
    pairs = list(itertools.permutations(range(n), 2))
    return {"gpus": n, "xgmi_links": len(xgmi), "full_xgmi_mesh": n > 1 and all(p in xgmi for p in pairs),
            "max_link_weight": max((v["weight"] for v in topo["links"].values()), default=0)}


def link_cost(topo: Optional[dict], a: int, b: int) -> float:
    """Relative cost of moving data a -> b (1 = direct xGMI link, larger = worse)."""
    if topo is None or a == b:
        return 1.0
    v = topo["links"].get((a, b))
    if v is None:
        return 8.0                 # no direct link: routed through a peer or the host
    return 1.0 if v["type"] == LINK_XGMI else 4.0


def order_stages(topo: Optional[dict], ranks: list) -> list:
    """Order a pipeline's ranks (first stays the driver) so consecutive stages sit on the
    cheapest links: greedy nearest neighbour, identity on a full mesh."""
    if topo is None or len(ranks) <= 2:
        return list(ranks)
    out, left = [ranks[0]], list(ranks[1:])
    while left:
        nxt = min(left, key=lambda r: (link_cost(topo, out[-1], r), left.index(r)))
        out.append(nxt)
        left.remove(nxt)
    return out
