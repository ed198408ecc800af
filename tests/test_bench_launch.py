"""CPU: bench.py's rank launch contract (StreamingJob.java:177 setParallelism).
`--gpus N` under a launcher must match WORLD_SIZE -- a mismatch exits non-zero before any torch
import.  The self-launch itself (bench.py --gpus 2 starting torch.distributed.run as its child)
runs on the GPU box: tests/test_a_gpu_multirank.py."""
import os
import subprocess
import sys

from conftest import ROOT


def _bench(args, **env):
    e = dict(os.environ)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=120)


def test_world_size_mismatch_is_refused():
    p = _bench(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr
    assert p.stdout == ""


def test_gpus_must_be_positive():
    e = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"], env=e, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2 and "--gpus must be >= 1" in p.stderr
