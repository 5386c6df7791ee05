"""Data-parallel correctness with the model in the loop (SURVEY §4 item 4,
§8e): two ranks (gloo, both on cuda:0 -- bench.py's RR_BENCH_ONE_DEVICE
mapping) each run the ResUNet unified step on half of a fixed batch with
per-replica BatchNorm under roadrestore.parallel.DataParallel.  The
all-reduced gradients must equal the average of two single-process
half-batch backward passes, and the parameters must stay identical across
ranks over three AdamW steps (tests/dp_worker.py does the checking).

The ranks are child processes started from this (GPU-initialised) process
with subprocess -- never an exec of this process."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, dtype):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RR_DP_DTYPE=dtype,
                   OMP_NUM_THREADS="4")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dp_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res = []
    for rc, out in outs:
        print(out[-3000:])
        assert rc == 0, out[-3000:]
        res.append(json.loads(out.strip().splitlines()[-1]))
    return res


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_dp_two_ranks_grads_and_params(dev, dtype):
    res = _run(2, dtype)
    assert all(r["pass"] for r in res), res
    assert res[0]["digest"] == res[1]["digest"]
