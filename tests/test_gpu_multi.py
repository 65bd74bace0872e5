"""world_size 2 on the GPU box: `bench.py --gpus 2` starts two ranks with
torch.distributed.run (device = LOCAL_RANK mod the visible devices, so both
share the one GPU of a test box), each tracks its own streams, and both
ranks' sampled streams of the timed trackers match the oracle."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def test_bench_two_ranks(tmp_path):
    detail = tmp_path / "detail.json"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--streams", "16", "--steps", "2",
           "--warmup", "1", "--loop", "8", "--secondary-steps", "0", "--stereo-steps", "0",
           "--rig-steps", "0", "--no-cpu-baseline", "--sweep", "0", "--isolated-steps", "0",
           "--detail", str(detail)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(ROOT))
    assert out.returncode == 0, out.stderr[-3000:]
    line = [x for x in out.stdout.splitlines() if x.startswith("{")][-1]
    c = json.loads(line)                       # the compact stdout record
    assert c["parity"]["pass"] is True and c["parity"]["headline_pass"] is True, c["parity"]
    r = json.loads(detail.read_text())         # the full report
    assert r["n_gpus"] == 2
    assert r["config"]["frames_per_step"] == 32
    assert r["value"] > 0
    par = r["parity"]
    assert par["all_ranks_pass"], par
    assert len(par["by_rank"]) == 2
    assert all(p["steps_checked"] == 3 for p in par["by_rank"])


def test_bench_lines_1024_streams_parity(tmp_path):
    """The lines workload timed at 1024 streams (the LSD scratch of every
    stream resident at once): the timed tracker's sampled streams 0, 512 and
    1023 match the oracle loop bit-exact (counts) / within POSE_TOL (pose)."""
    detail = tmp_path / "detail.json"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--workload", "lines", "--streams", "1024",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--sweep", "0",
           "--isolated-steps", "0", "--ingress-steps", "0", "--detail", str(detail)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(ROOT))
    assert out.returncode == 0, out.stderr[-3000:]
    c = json.loads([x for x in out.stdout.splitlines() if x.startswith("{")][-1])
    assert c["parity"]["pass"] is True and len(json.dumps(c)) < 8192
    r = json.loads(detail.read_text())
    assert r["config"]["streams_per_gpu"] == 1024 and r["tracking"]["mean_lines"] > 50
    par = r["parity"]
    assert par["pass"] and par["streams"] == [0, 512, 1023] and par["steps_checked"] == 3, par
