"""CPU: bench.py's multi-rank path — `--gpus 2` launches two ranks
through torch.distributed.run as a child process, the ranks meet over gloo,
walk-step counts are summed over ranks, the max-over-ranks time is taken and
the all-gather of the emitted rows is checked byte-for-byte on rank 0.  The
rows are synthetic (`--plumbing-check`: no GPU here); the GPU test
`test_n2v_gpu.py::test_bench_two_ranks_gloo_on_gpu` runs the same path with
real walks."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=env,
                       cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("ranks,limit", [(2, None), (2, 200_000), (4, None)])
def test_bench_multi_rank_plumbing(ranks, limit):
    steps, scale, L, nw = 3, 8, 80, 10
    env = {"GW_BENCH_GATHER_LIMIT": str(limit)} if limit else None
    rc, res, err = _run(["--gpus", str(ranks), "--plumbing-check", "--scale", str(scale), "--steps", str(steps),
                         "--warmup", "1"], env)
    assert rc == 0, err[-2000:]
    assert res["ranks"] == ranks and res["backend"] == "gloo"
    assert res["n_gpus"] == 0 and "rehearsal" in res  # no GPU: never reported as a GPU count
    B = nw * (1 << scale)
    assert res["config"]["walks_per_step"] == ranks * B
    assert res["walk_steps"] == ranks * steps * B * (L - 1)
    g = res["allgather"]
    assert g["check_last_rank_block_identical"] is True and res["allgather_all_ranks_ok"] is True
    assert g["gathered_bytes_per_step_per_rank"] == (ranks - 1) * B * L * 4
    if limit is not None:
        assert g["mode"] == f"ring of {limit // (ranks * L * 4)}-row chunks"
    else:
        assert g["mode"] == "whole"
    # SURVEY §8e's alternative exchange: every rank writes its own shard to host memory
    h = res["host_shard"]
    assert h["check_host_rows_equal_device_rows"] is True
    assert h["bytes_per_step_per_rank"] == B * L * 4 and h["seconds"] > 0


@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_config4_strong_plumbing(ranks):
    """Config 4's BASELINE shape (the r=10 workload split over
    the GPUs, walks all-gathered): shard_range shards (uneven by one walk,
    padded for the collective), the summed walk-steps equal ONE pass of the
    fixed workload per step whatever the rank count, and the gathered block
    of the last rank equals rank 0's recomputation of it."""
    steps, scale, L, r = 2, 8, 80, 10
    rc, res, err = _run(["--gpus", str(ranks), "--plumbing-check", "--config", "4", "--scale", str(scale),
                         "--steps", str(steps), "--warmup", "1"])
    assert rc == 0, err[-2000:]
    total = r * (1 << scale)
    assert res["scaling"] == "strong" and res["ranks"] == ranks
    assert res["config"]["walks_per_step"] == total and "strong" in res["config"]["parallelism"]
    assert res["walk_steps"] == steps * total * (L - 1)
    g = res["allgather"]
    assert g["check_last_rank_block_identical"] is True and res["allgather_all_ranks_ok"] is True
    rows = -(-total // ranks)
    assert g["gathered_bytes_per_step_per_rank"] == (ranks - 1) * rows * L * 4
    h = res["host_shard"]  # the shard written to host memory instead of gathered
    assert h["check_host_rows_equal_device_rows"] is True
    assert total // ranks * L * 4 <= h["bytes_per_step_per_rank"] <= rows * L * 4


@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_config5_rows_allgather_plumbing(ranks):
    """Config 5's exchange (k x (int32 + fp64) per source): the
    round-robin source shards' top-100 rows all-gathered to every rank, each
    received block checked against its sender's checksum."""
    scale, K = 8, 100
    rc, res, err = _run(["--gpus", str(ranks), "--plumbing-check", "--config", "5", "--scale", str(scale),
                         "--steps", "2"])
    assert rc == 0, err[-2000:]
    assert res["scaling"] == "strong" and res["ranks"] == ranks
    g = res["allgather"]
    assert g["check_blocks_match_sender_checksums"] is True
    rows = -(-(1 << scale) // ranks)
    assert g["gathered_bytes_per_step_per_rank"] == (ranks - 1) * rows * K * 12
    h = res["host_shard"]  # each rank's own rows to host memory, no exchange
    assert h["check_host_rows_equal_device_rows"] is True
    assert (1 << scale) // ranks * K * 12 <= h["bytes_per_rank"] <= rows * K * 12


def test_bench_rank_count_mismatch_is_refused():
    rc, res, err = _run(["--gpus", "2", "--plumbing-check"], {"WORLD_SIZE": "1"}, timeout=120)
    assert rc == 2 and res is None
    assert "WORLD_SIZE=1" in err
