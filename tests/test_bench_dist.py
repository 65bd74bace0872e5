"""The N>1 path of bench.py on CPU (gloo, world size 2): the max-over-ranks
wall time, the per-rank parity gather, the `--gpus N` launcher command, and
a 2-rank torchrun of bench's own rank bootstrap (env contract: RANK /
LOCAL_RANK / WORLD_SIZE, MASTER_ADDR 127.0.0.1)."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    t = bench.max_over_ranks(dist, 1.0 + rank)        # rank 1 is the slow one
    par = bench.gather_parity(dist, world, {"pass": rank == 0 or q is None, "rank": rank})
    q.put((rank, t, par))
    dist.destroy_process_group()


def test_max_time_and_parity_gather_ws2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, t, par in res:
        assert t == 2.0                                  # the max over ranks
        assert [p["rank"] for p in par["by_rank"]] == [0, 1]
        assert par["all_ranks_pass"] is False            # rank 1 reported a failure


def test_gpus_flag_builds_torchrun_command():
    import bench
    cmd = bench.torchrun_cmd(8, ["--gpus", "8", "--steps", "3"], 29555)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")


def test_torchrun_two_ranks_env_contract():
    """torch.distributed.run with 2 ranks on CPU: each rank sees the env that
    bench.py reads and reaches the gloo barrier."""
    tmp = Path(os.environ.get("TMPDIR", "/tmp"))
    tag = f"orbpl_ws2_{os.getpid()}"
    # each rank writes its own file (the ranks' shared stdout can interleave)
    code = ("import os, torch.distributed as d; d.init_process_group('gloo'); d.barrier(); "
            f"open(os.path.join({str(tmp)!r}, '{tag}_' + os.environ['RANK'] + '.txt'), 'w').write("
            "' '.join(['rank', os.environ['RANK'], os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE']]))")
    script = tmp / f"{tag}.py"
    script.write_text(code)
    outs = [tmp / f"{tag}_{r}.txt" for r in range(2)]
    try:
        out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                              "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port",
                              str(_port()), str(script)], capture_output=True, text=True,
                             timeout=180)
        assert out.returncode == 0, out.stderr[-2000:]
        lines = [o.read_text() for o in outs]
    finally:
        script.unlink()
        for o in outs:
            o.unlink(missing_ok=True)
    assert lines == ["rank 0 0 2", "rank 1 1 2"]


def _vocab_rank(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    sys.path.insert(0, str(ROOT / "tests"))
    from _pkg import load_pkg
    load_pkg()
    import orbpl.synth as synth
    rng = np.random.default_rng(5 + rank)
    docs = [rng.integers(0, 256, (200, 32), dtype=np.uint8) for _ in range(3)]
    tree = synth.vocabulary_tree(docs, k=4, L=3, seed=2) if rank == 0 else None
    tree = bench.share_tree(tree, dist)
    w, n_docs, backend = bench.shared_idf(synth, tree, docs, dist)
    q.put((rank, tree["desc"].tobytes(), w, n_docs, backend,
           [d.tobytes() for d in docs]))
    dist.destroy_process_group()


def test_shared_vocabulary_ws2():
    """Rank 0's vocabulary tree reaches rank 1 (broadcast) and the IDF weights
    from the all-reduced document counts equal those of one process holding
    every rank's documents."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "tests"))
    from _pkg import load_pkg
    load_pkg()
    import orbpl.synth as synth
    import bench
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_vocab_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (_, t0, w0, n0, b0, d0), (_, t1, w1, n1, b1, d1) = res
    assert t0 == t1 and np.array_equal(w0, w1) and n0 == n1 == 6 and b0 == "gloo"
    docs = [np.frombuffer(b, np.uint8).reshape(-1, 32) for b in d0 + d1]
    rng = np.random.default_rng(5)
    tree = synth.vocabulary_tree([rng.integers(0, 256, (200, 32), dtype=np.uint8)
                                  for _ in range(3)], k=4, L=3, seed=2)
    assert tree["desc"].tobytes() == t0
    w, n, _ = bench.shared_idf(synth, tree, docs, None)
    assert n == 6 and np.array_equal(w, w0)
    assert (w0 > 0).sum() > 10


def test_compact_line_fits_the_driver_tail():
    """bench.py's last stdout line carries the contract's keys, the dominant
    kernel's roofline, the CPU baseline, the parity verdict and the leg
    summary within COMPACT_MAX bytes (round 5's 22.5 KB line was unparsed);
    input: the full round-5 record committed under profiles/r05/."""
    import json
    import bench
    full = json.loads((Path(__file__).resolve().parents[1] / "profiles" / "r05" /
                       "bench_r05_h_default.json").read_text().strip().splitlines()[-1])
    c = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(c)
    assert "\n" not in s and len(s) <= bench.COMPACT_MAX
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in c
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel"):
        assert k in c["roofline"]
    assert c["cpu_baseline"]["cores"] and c["cpu_baseline"]["reference_faithful_ms"]
    assert c["parity"]["pass"] is True
    assert {"points", "secondary", "stereo", "rig", "ingress", "batch1_ms"} <= set(c["summary"])


def test_compact_line_gathered_parity():
    """With ranks > 1 the headline parity is the gathered {all_ranks_pass,
    by_rank} report: the compact line's verdict follows all_ranks_pass."""
    import bench
    base = {"metric": "m", "value": 1.0, "unit": "frames/s", "n_gpus": 2, "steps": 1, "warmup": 1,
            "ms_per_step": 1.0, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic", "config": {}, "roofline": None,
            "cpu_baseline": None, "summary": {}}
    for ok in (True, False):
        out = dict(base, parity={"all_ranks_pass": ok,
                                 "by_rank": [{"pass": True, "pose_tol": 1e-4},
                                             {"pass": ok, "pose_tol": 1e-4}]})
        c = bench.compact_line(out, "d.json")
        assert c["parity"]["pass"] is ok and c["parity"]["headline_pass"] is ok
        assert c["parity"]["pose_tol"] == 1e-4
