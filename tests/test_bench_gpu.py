"""GPU: bench.py end to end on small graphs — one rank, and two ranks on the
one GPU of the test box over gloo (GW_DIST_BACKEND=gloo: RCCL refuses two ranks
on one device), which exercises the launcher, the weak-scaling walk blocks, the
max-over-ranks timing and the all-gather check with real HIP walks."""
import json
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--scale", "12", "--steps", "2", "--warmup", "1", "--secondary", "none", "--no-cpu-baseline"]


def _run(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, "-u", BENCH] + args, capture_output=True, text=True, timeout=timeout,
                       env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.gpu
def test_bench_one_rank_small():
    rc, res, err = _run(SMALL)
    assert rc == 0, err[-3000:]
    assert res["n_gpus"] == 1 and res["ranks"] == 1 and res["value"] > 0
    r = res["roofline"]
    assert r["units_per_launch"] * 2 == res["walk_steps"]
    assert r["random_line_roofline"]["calibrated_peak_lines_per_s"] > 1e10


@pytest.mark.gpu
def test_bench_two_ranks_gloo_on_gpu():
    rc, res, err = _run(["--gpus", "2"] + SMALL, {"GW_DIST_BACKEND": "gloo"})
    assert rc == 0, err[-3000:]
    assert res["ranks"] == 2 and res["n_gpus"] == 1 and "rehearsal" in res
    n = int(res["config"]["walks_per_step"]) // 20  # 10 walks/node per rank, 2 ranks
    # R-MAT is undirected with no isolated starts: every walk has all 80 positions
    assert res["walk_steps"] == 2 * 2 * 10 * n * 79
    assert res["allgather"]["check_last_rank_block_identical"] is True
    assert res["allgather_all_ranks_ok"] is True
    h = res["host_shard"]  # gw_n2v_walks_host into pinned memory, rows equal the device walks
    assert h["check_host_rows_equal_device_rows"] is True and h["host_memory"] == "pinned"
    assert h["bytes_per_step_per_rank"] == 10 * n * 80 * 4


@pytest.mark.gpu
def test_bench_config4_shape_small():
    # config 4's sampler and p/q (rejection, p=1, q=0.5) on a small R-MAT
    rc, res, err = _run(["--config", "4"] + SMALL)
    assert rc == 0, err[-3000:]
    assert res["sampler"] == "rejection" and res["config"]["baseline_config"] == 4
    assert res["value"] > 0 and 1.0 <= res["rejection_trials_per_step"] < 3.0


@pytest.mark.gpu
def test_bench_config4_strong_two_ranks_gloo_on_gpu():
    """Config 4's BASELINE shape with real walks: the fixed r=10 workload
    split over 2 ranks (strong scaling), then all-gathered; the last rank's
    gathered block equals rank 0's own recomputation of it."""
    rc, res, err = _run(["--gpus", "2", "--config", "4"] + SMALL, {"GW_DIST_BACKEND": "gloo"})
    assert rc == 0, err[-3000:]
    assert res["scaling"] == "strong" and res["ranks"] == 2
    total = res["config"]["walks_per_step"]
    assert res["walk_steps"] <= 2 * total * 79 and res["walk_steps"] > 0
    assert res["allgather"]["check_last_rank_block_identical"] is True and res["allgather_all_ranks_ok"] is True
    assert res["end_to_end"]["prepare_s"] >= 0 and res["end_to_end"]["value"] > 0
    h = res["host_shard"]
    assert h["check_host_rows_equal_device_rows"] is True and h["value"] > 0


@pytest.mark.gpu
def test_bench_config5_two_ranks_rows_allgather_gloo_on_gpu():
    """Config 5 (TopSim top-100) on a 200k-vertex Java R-MAT over 2 ranks: the
    round-robin source shards' rows all-gathered, blocks checked against the
    senders' checksums."""
    rc, res, err = _run(["--gpus", "2", "--config", "5", "--p10m-vertices", "200000", "--no-cpu-baseline"],
                        {"GW_DIST_BACKEND": "gloo"})
    assert rc == 0, err[-3000:]
    assert res["scaling"] == "strong" and res["ranks"] == 2 and res["value"] > 0
    assert res["allgather"]["check_blocks_match_sender_checksums"] is True
    h = res["host_shard"]
    assert h["check_host_rows_equal_device_rows"] is True and h["value"] > 0


@pytest.mark.gpu
def test_bench_config3_sweep_small():
    """The config-3 sweep (Test_u_u_TopSim_singleSample's loop) at two SAMPLEs on
    moreno and arxiv: one point per (graph, SAMPLE), each naming the kernel it
    dispatched with its registers / scratch, the timed dispatch's ordinal for
    the PMC passes, and a CPU oracle baseline where asked."""
    rc, res, err = _run(["--scale", "10", "--steps", "1", "--warmup", "0", "--no-walk10m", "--no-simrank",
                         "--no-rmat24", "--no-p10m", "--no-p10m-stretch", "--no-arxiv", "--topsim-graphs", "moreno",
                         "--config3-graphs", "moreno,arxiv", "--config3-samples", "1000,5000",
                         "--config3-cpu-samples", "1000", "--config3-cpu-seconds", "0.5", "--cpu-seconds", "0.5"])
    assert rc == 0, err[-3000:]
    sw = res["secondary"]["topsim_config3"]
    pts = sw["points"]
    assert [(p["graph"], p["sample"]) for p in pts] == [("moreno", 1000), ("moreno", 5000), ("arxiv", 1000),
                                                        ("arxiv", 5000)]
    for p in pts:
        assert p["value"] > 0 and p["kernel"].startswith("k_topsim") and p["config"]["step"] == 5
        assert p["kernel_attrs"]["vgprs"] > 0 and p["kernel_attrs"]["scratch_bytes_per_lane"] >= 0
        m = p["roofline"]["pmc_match"]
        assert m["nth"][0] >= 0 and re.match(m["kernel"], p["kernel"])
        assert (p["cpu_baseline"] is not None) == (p["sample"] == 1000)
    assert pts[0]["kernel"] == "k_topsim_2wg<5, 0>"  # moreno: the dense LDS row at two workgroups per CU
    assert pts[2]["kernel"] == "k_topsim_pipe<5>"    # arxiv, SAMPLE <= 2048: the pipelined hash kernel
    assert pts[3]["kernel"] == "k_topsim_2wg<5, 2>"  # arxiv 5000: W/E < 16 keeps the unpipelined kernel
    # the moreno line of secondary.topsim is NOT a second run of the sweep's point at another SAMPLE
    assert res["secondary"]["topsim"]["config"]["sample"] == 10000
