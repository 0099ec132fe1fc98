"""bench.py's multi-GPU launch contract (CPU): ``--gpus N`` either runs as one of N ranks under
a launcher with WORLD_SIZE = N, spawns N ranks itself, or refuses -- it never prints an
N = 1 record for an N-GPU request."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import bench  # noqa: E402


def test_plan_single_gpu_without_launcher():
    assert bench.launch_plan(1, {}, 1) == ("run", 1, 0, 0)
    assert bench.launch_plan(1, {}, 8) == ("run", 1, 0, 0)


def test_plan_spawns_n_ranks_without_launcher():
    for n in (2, 4, 8):
        assert bench.launch_plan(n, {}, 8) == ("spawn", n)


def test_plan_runs_as_a_launcher_rank():
    env = {"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"}
    assert bench.launch_plan(8, env, 8) == ("run", 8, 5, 5)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, 1) == ("run", 1, 0, 0)


@pytest.mark.parametrize("gpus,env,devs", [
    (2, {}, 1),                                                  # --gpus 2 on a 1-GPU box
    (8, {}, 0),                                                  # no GPU at all
    (1, {}, 0),
    (2, {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"}, 8),  # launcher disagrees with --gpus
    (4, {"WORLD_SIZE": "1"}, 8),
    (2, {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}, 1),  # local rank without a device
    (2, {"WORLD_SIZE": "2", "RANK": "2", "LOCAL_RANK": "0"}, 2),  # rank out of range
    (0, {}, 8),
])
def test_plan_refuses(gpus, env, devs):
    assert bench.launch_plan(gpus, env, devs)[0] == "refuse"


def _run_bench(args, extra_env):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env)
    return subprocess.run([sys.executable, os.path.join(HERE, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


@pytest.mark.skipif(__import__("torch").cuda.device_count() >= 2, reason="needs a box with fewer than 2 GPUs")
def test_gpus_2_without_two_devices_fails_loudly():
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {})
    assert r.returncode == 2, r.stderr
    assert "--gpus 2" in r.stderr and r.stdout == ""


def test_spawned_ranks_rendezvous_and_rank0_prints_once():
    """The self-launch path end to end on CPU: N children with WORLD_SIZE/RANK set, one gloo
    all-reduce across them, exactly one JSON line (rank 0's)."""
    r = _run_bench(["--gpus", "3", "--launch-probe"], {})
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]   # gloo logs its own lines
    assert len(lines) == 1 and '"n_gpus": 3' in lines[0], r.stdout
    # the N > 1 line's fields, assembled over the process group (bench.multi_gpu_fields)
    m = __import__("json").loads(lines[0])["multi_gpu"]
    assert m["world_size_process_group"] == 3 and m["backend"] == "gloo"
    assert m["rank_matrix_ms"] == {"min": 1.0, "max": 3.0} and m["rank_scan_ms"] == {"min": 2.0, "max": 4.0}
    assert m["allgather"]["bytes_per_rank"] == 1234 and m["allgather"]["bytes_total"] == 3 * 1234
    assert abs(m["allgather"]["ms_max_over_ranks"] - 0.15) < 1e-12
    # the whole-corpus CPU restatement, distributed over the ranks' shards and merged on rank 0, equals
    # the single-index oracle (ties straddle a shard boundary)
    assert m["sample_check"]["queries"] == 8 and m["sample_check"]["top10_identical"] == 1.0


def test_world_size_mismatch_is_refused():
    r = _run_bench(["--gpus", "2", "--steps", "1"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=3" in r.stderr and r.stdout == ""


def test_visible_gpus_counts_kfd_gpu_nodes_without_hip(tmp_path):
    """The launcher parent counts devices from the KFD topology (CPU nodes have simd_count 0), narrowed
    by the *_VISIBLE_DEVICES variables, without a HIP call."""
    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simds}\nmem_banks_count 1\n")
    assert bench.visible_gpus({}, str(tmp_path)) == 3
    assert bench.visible_gpus({"HIP_VISIBLE_DEVICES": "0,2"}, str(tmp_path)) == 2
    assert bench.visible_gpus({"ROCR_VISIBLE_DEVICES": "1"}, str(tmp_path)) == 1


def test_shard_ranges_cover_every_row_once():
    from vectorragquantization_amd import synth
    for n in (1000, 6400, 100_000_000, 12_345_677):
        for world in range(1, 9):
            rs = [synth.shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
