"""The product's row-sharded search across two real processes on the one GPU of the box
(tests/_gpu_dist_worker.py): each rank runs the HIP kernels on its own shard, the packed per-shard
candidates cross a real process boundary through one all-gather (gloo, host-staged), and the merge
kernel's output must equal the single-index search bit for bit -- config 4 (vrq_search3 SHARD ->
vrq_merge_shards) and config 5 (vrq_gemm_topk with row offsets -> merge_topk_shards)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.timeout(240)
def test_two_process_sharded_search_equals_single_index(tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    res = tmp_path / "result.txt"
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), VRQ_DIST_RESULT=str(res), VRQ_DIST_ROWS="1000000")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "_gpu_dist_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=200)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-3000:] for o in outs)
    assert res.read_text() == "OK"
