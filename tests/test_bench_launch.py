"""bench.py's launcher (CPU, gloo): `--gpus N` without torch.distributed.run starts N ranks itself,
each rank joins a world of exactly N, and a world that does not match --gpus is an error."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", **extra)
    return env


def _run(args, **extra):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=_env(**extra), cwd=ROOT)


def test_gpus_n_spawns_n_ranked_workers():
    r = _run(["--gpus", "3", "--check-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # only rank 0 prints
    d = json.loads(lines[0])
    assert d["world_size"] == 3 and d["n_gpus"] == 3 and d["backend"] == "gloo"
    assert sorted(x[0] for x in d["ranks"]) == [0, 1, 2]
    assert all(rk == lr for rk, lr, _ in d["ranks"])     # one node: local rank == rank


def test_single_process_default():
    r = _run(["--check-launch"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["world_size"] == 1 and d["ranks"] == [[0, 0, -1]]


def test_world_mismatch_fails():
    r = _run(["--gpus", "2", "--check-launch"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "--gpus 2" in r.stderr


def test_strong_scaling_plan():
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse_args(["--gpus", "8", "--global-batch", "4096"])
    plans = [bench.batch_plan(a, 8, r, 512) for r in range(8)]
    assert all(p["B"] == 512 and p["scaling"] == "strong" and p["B_global"] == 4096 for p in plans)
    assert plans[3]["lo"] == 1536 and plans[3]["hi"] == 2048
    a = bench.parse_args(["--global-batch", "4096"])
    assert bench.batch_plan(a, 1, 0, 512)["B"] == 4096
    a = bench.parse_args(["--gpus", "4"])
    p = bench.batch_plan(a, 4, 2, 512)
    assert p["B"] == 512 and p["B_global"] == 2048 and p["scaling"] == "weak"


def test_every_workload_is_registered():
    """Each --workload choice parses (row †g's segno_train included)."""
    sys.path.insert(0, ROOT)
    import bench
    for wl in ("egno", "segno", "segno_gravity", "egno_train", "segno_train", "egno_rollout", "sim_charged"):
        assert bench.parse_args(["--workload", wl]).workload == wl
