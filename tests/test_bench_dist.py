"""The N>1 bench path (replicas: barrier + max-over-ranks timer, no data-path collective),
rehearsed with world_size-2 gloo on CPU."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    import time

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ws, r, local = bench.dist_env()
    assert (ws, r, local) == (world, rank, rank)
    barrier, reduce_max = bench.make_collectives(torch, dist)
    # rank 1 is slower: the reported time must be the max over ranks
    dt = bench.timed_region(lambda: time.sleep(0.05 + 0.1 * rank), barrier, lambda: None, reduce_max)
    q.put((rank, dt))
    dist.destroy_process_group()


def test_timed_region_reports_max_over_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res = dict(q.get() for _ in range(2))
    assert res[0] == res[1]            # every rank reports the same (max) time
    assert 0.15 <= res[0] < 1.0        # the slow rank's 0.15 s dominates


def test_single_process_collectives_are_identity():
    import bench

    barrier, reduce_max = bench.make_collectives(torch, None)
    barrier()
    assert reduce_max(1.5) == 1.5
    assert bench.gather(None, "x") == ["x"]


_RANK_SCRIPT = r"""
import os, sys, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
import bench
ws, rank, local = bench.dist_env()
assert ws == 2 and rank == local and os.environ["MASTER_ADDR"] == "127.0.0.1", (ws, rank, local)
dist.init_process_group("gloo")
got = bench.gather(dist, rank * 10)
assert got == [0, 10], got
dist.destroy_process_group()
sys.exit(int(sys.argv[2]) if rank == 1 else 0)
"""


def test_launcher_starts_one_rank_per_gpu(tmp_path):
    """bench.py --gpus N outside torchrun: N rank processes with RANK/LOCAL_RANK/WORLD_SIZE and a
    127.0.0.1 rendezvous, gloo group, exit status propagated."""
    import sys

    import bench

    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env_ws = os.environ.pop("WORLD_SIZE", None)
    try:
        assert bench.launch_replicas(2, [repo, "0"], count_devices=lambda: 2, script=str(script)) == 0
        assert bench.launch_replicas(2, [repo, "3"], count_devices=lambda: 2, script=str(script)) == 3
    finally:
        if env_ws is not None:
            os.environ["WORLD_SIZE"] = env_ws


def test_launcher_refuses_missing_devices(capsys):
    import bench

    assert bench.launch_replicas(8, [], count_devices=lambda: 1) == 2
    assert "--gpus 8 needs 8 visible GPUs, found 1" in capsys.readouterr().err


def test_launcher_refuses_when_device_count_unknown(capsys):
    """The launcher never falls back to counting devices in its own process (that would initialise
    HIP in the parent that spawns the ranks): a failed probe is exit 2 with a message."""
    import bench

    called = []
    assert bench.launch_replicas(2, [], count_devices=lambda: None, script="/nonexistent") == 2
    assert "could not count the visible GPUs" in capsys.readouterr().err
    assert not called


def test_device_probe_runs_in_a_child(monkeypatch):
    """probe_device_count() answers from a child process; a broken interpreter gives None."""
    import bench

    n = bench.probe_device_count()
    assert n == torch.cuda.device_count()
    assert bench.probe_device_count(python="/nonexistent/python") is None


_SLOW_RANK = r"""
import os, sys, time
rank = int(os.environ["RANK"])
if rank == 0:
    sys.exit(5)          # dies before any rendezvous
time.sleep(120)          # would wait in the rendezvous for the default timeout
"""


def test_launcher_ends_the_job_at_the_first_failure(tmp_path):
    import time

    import bench

    script = tmp_path / "slow.py"
    script.write_text(_SLOW_RANK)
    env_ws = os.environ.pop("WORLD_SIZE", None)
    try:
        t0 = time.time()
        assert bench.launch_replicas(3, [], count_devices=lambda: 3, script=str(script)) == 5
        assert time.time() - t0 < 30
    finally:
        if env_ws is not None:
            os.environ["WORLD_SIZE"] = env_ws


def test_bench_gpus2_fails_loudly_without_devices():
    """The driver's `python bench.py --gpus 2` on a box with fewer GPUs exits non-zero with a message."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if torch.cuda.device_count() >= 2:
        pytest.skip("this host has >= 2 GPUs")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--quick"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "--gpus 2 needs 2 visible GPUs" in r.stderr


def test_cpu_share_respects_quota(monkeypatch):
    import bench

    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    use, aff, _ = bench.cpu_share()
    assert use == min(3, aff)


def test_work_accounting():
    import bench

    assert bench.call_flops(1, 4, 1024, 1024) == 1073741824
    assert bench.call_bytes(1, 4, 1024, 1024) == 2097152
    assert bench.call_bytes(1, 4, 1024, 1024, out_bytes=4) == 2621440


def test_bench_refuses_world_size_mismatch():
    """Under a torchrun environment, --gpus must equal WORLD_SIZE (checked before any GPU call)."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29555")
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "1", "--quick"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2
    assert "--gpus 1 but WORLD_SIZE=2" in r.stderr


def test_claim_stdout_keeps_only_the_json_line():
    """With several ranks, C-level writes to fd 1 (gloo's connection messages) land on stderr and
    only the line written to the claimed stream reaches stdout."""
    code = (
        "import os, sys; sys.path.insert(0, %r); import bench\n"
        "out = bench.claim_stdout(4)\n"
        "os.write(1, b'[Gloo] Rank 0 is connected to 3 peer ranks\\n')\n"
        "print('noise from python')\n"
        "print('{\"metric\": 1}', file=out, flush=True)\n"
    ) % REPO
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == '{"metric": 1}'
    assert "Gloo" in r.stderr and "noise from python" in r.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_hardware():
    """The N>1 path on the GPU box: `BENCH_SHARE_DEVICE=1 bench.py --gpus 2 --quick` (two rank
    processes sharing the one GPU, gloo group, per-rank rates, cross-rank output digest). Exactly one
    JSON line on stdout."""
    import json

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_SHARE_DEVICE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--quick", "--steps", "200",
                        "--warmup", "20"], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert len(d["per_rank_calls_per_s"]) == 2 and all(v > 0 for v in d["per_rank_calls_per_s"])
    assert d["outputs_bitwise_identical_across_ranks"] is True
