"""GPU, world size 2 on one device: bench.py's N > 1 code paths executed end to end (VERDICT r02
"Next round" item 5) -- the kNN headline path (cell-column shards, device records written at
pipeline depth 3 on two streams, batched all-gather of the records, gf_knn_merge_dev_batch with
GF_MERGE_FOREIGN_KEYS, gf_ctx_join / gf_ctx_fork ordering around each exchange) and the C5
sliding path (pane engine per rank, window records all-gathered and merged).  Two ranks are
launched with torch.distributed.run on the gloo backend (the all-gather goes through host
memory; the RCCL backend is the driver's multi-GPU run), and each bench run asserts its merged
records against the oracle on the whole window (every rank's band regenerated from its seed):
bench.py "verified_vs_oracle", tools/bench_workloads.py "verified_vs_whole_window_and_oracle".
Anchor: PointPointKNNQuery.java:198-200 (the windowAll funnel the exchange replaces).

The file is named to run first: the ranks are started before this pytest process makes any GPU
call (a process that has initialised the GPU must not fork + exec children on this pool)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_two_ranks(extra, launcher=False):
    """bench.py --gpus 2 as the user runs it: bench.py itself starts the two ranks
    (torch.distributed.run as its child).  launcher=True: the driver's form, torchrun in front."""
    import torch

    assert not torch.cuda.is_initialized(), "start the ranks before this process touches the GPU"
    pre = [sys.executable]
    if launcher:
        pre += ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port())]
    cmd = pre + [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--no-cpu-baseline"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-6000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("pipeline,launcher", [(3, False), (2, False), (4, False), (3, True)])
def test_knn_two_ranks_verified(pipeline, launcher):
    line = _run_two_ranks(["--points", "400000", "--steps", "9", "--warmup", "3", "--windows", "4",
                           "--exchange-batch", "2", "--pipeline", str(pipeline)], launcher=launcher)
    assert line["n_gpus"] == 2 and line["verified_vs_oracle"] is True
    assert line["config"]["points_per_window"] == 800_000


@pytest.mark.timeout(900)
def test_knn_two_ranks_string_objids_verified():
    """String objIDs (each rank interns "veh%09d" into its own dictionary): the exchange attaches
    the Strings (gf_knn_attach_strings), all-gathers the string records and merges them by String
    on the device (gf_knn_merge_dev_strings) -- verified against the oracle on the whole window."""
    line = _run_two_ranks(["--points", "400000", "--steps", "9", "--warmup", "3", "--windows", "4",
                           "--exchange-batch", "2", "--pipeline", "3", "--string-objids"])
    assert line["n_gpus"] == 2 and line["verified_vs_oracle"] is True
    assert line["config"]["objid"].startswith("dictionary Strings")


@pytest.mark.timeout(900)
def test_sliding_two_ranks_verified():
    line = _run_two_ranks(["--workload", "sliding", "--points", "2000000", "--steps", "7", "--warmup", "3",
                           "--windows", "3", "--exchange-batch", "2"])
    assert line["n_gpus"] == 2 and line["verified_vs_whole_window_and_oracle"] is True
