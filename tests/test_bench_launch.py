"""bench.py's rank launcher (CPU, gloo): `python bench.py --gpus N` starts N
ranks through torch.distributed.run as a child process, and a rank whose
WORLD_SIZE disagrees with --gpus refuses to run.  --dry-run skips all
device work, so this runs without a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TORCHELASTIC_RUN_ID", "MASTER_PORT")}
    env.update(kw)
    return env


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # exactly one JSON line, from rank 0
    return json.loads(lines[0])


def test_gpus2_launches_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=240, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 2 and d["dry_run"] is True
    assert d["ranks"] == [0, 1]
    assert len(set(d["pids"])) == 2 and os.getpid() not in d["pids"]
    assert d["all_ranks_ok"] and d["scaling"] == "weak"
    assert d["bytes_per_step"] == 2 * 1024 * (128 << 20)  # C3: 1024 blocks per GPU


def test_gpus2_c4_strong_split():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--config", "C4"], capture_output=True,
                       text=True, timeout=240, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["bytes_per_step"] == 512 * (128 << 20)  # 64 GiB for the node


def test_gpus1_stays_in_process():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 1 and d["ranks"] == [0] and len(d["pids"]) == 1


def test_world_size_mismatch_refused():
    """Under torchrun with WORLD_SIZE=3, --gpus 2 must fail before any work."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0", TORCHELASTIC_RUN_ID="x"),
                       cwd=ROOT)
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr
