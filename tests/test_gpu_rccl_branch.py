"""bench.py's N>1 branch over RCCL, run at world size 1 on the one-GPU box.

The driver's multi-GPU bench is the only place bench.py's RCCL branch
(`init_process_group("nccl", device_id=...)`, the barriers, the device-tensor
`dist.gather` of `tiles.assemble`, the float64 / int64 `all_reduce`s of the
per-rank timings and event counters) would otherwise execute. With
IPT_BENCH_FORCE_DIST=1 bench.py builds that process group and runs every one
of those collectives with one rank, launched the way the driver launches it
(`torch.distributed.run`, 127.0.0.1 rendezvous), and `--verify` re-renders the
frame unsharded and compares the assembled one bit for bit. Two ranks cannot
share one GPU under RCCL, so the N = 2 / 4 rehearsals stay on gloo
(test_multigpu_gloo.py, bench.py IPT_BENCH_SHARE_GPU=1).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_bench_rccl_branch_single_rank():
    env = dict(os.environ, IPT_BENCH_FORCE_DIST="1")
    env.pop("IPT_BENCH_SHARE_GPU", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "bench.py"),
           "--gpus", "1", "--config", "c2", "--width", "96", "--height", "80", "--spp-per-step", "2",
           "--steps", "2", "--warmup", "1", "--cpu-seconds", "0", "--verify"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["value"] > 0
    # the assembled frame (one RCCL gather) == the unsharded re-render
    assert d["verify_whole_frame_bit_exact"] is True
    # the per-rank rows came through the RCCL all-reduces
    assert d["ranks"] and d["ranks"][0]["paths"] == 96 * 80 * 2 * 2
    assert "frame_end" in d
