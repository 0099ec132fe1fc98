"""Debug dump of the K1s pass (diagnostic build -DVRQ_K1S_DEBUG): workgroup 0, wave 0, row set 0."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from vectorragquantization_amd import _native as N  # noqa: E402

lib = N._open(sys.argv[1], sys.argv[1])
dev = torch.device("cuda", 0)
rng = np.random.default_rng(5)
n, nq, K = 131072, 512, 100
codes = rng.integers(0, 256, (n, 128), dtype=np.uint8)
qb = rng.integers(0, 256, (nq, 128), dtype=np.uint8)
c_t, q_t = torch.from_numpy(codes).to(dev), torch.from_numpy(qb).to(dev)
ws = torch.zeros((lib.vrq_search3_workspace_size(n, 1024, nq, K),), dtype=torch.uint8, device=dev)
st = N.stream_handle(dev)
base = N.VRQ_SEARCH_PHASE1_ONLY | N.VRQ_SEARCH_SCAN_MFMA
N.check(lib.vrq_search3_scan(N.ptr(c_t), n, 1024, N.ptr(q_t), nq, K, base | N.VRQ_SCAN_STAGE_PREFIX, N.ptr(ws),
                             ws.numel(), st), "prefix")
torch.cuda.synchronize()
ws[:5 * 4096 * 4].zero_()
N.check(lib.vrq_search3_scan(N.ptr(c_t), n, 1024, N.ptr(q_t), nq, K, base | N.VRQ_SCAN_STAGE_MATRIX, N.ptr(ws),
                             ws.numel(), st), "matrix")
torch.cuda.synchronize()
d = ws[:5 * 4096 * 4].cpu().numpy().view(np.uint32)
w32 = codes.view(np.uint32)  # [n, 32]
pc_rows = np.unpackbits(codes, axis=1).sum(1)
pcq = np.unpackbits(qb, axis=1).sum(1)
l = np.arange(64)
print("pc  (lanes 0..31, rows 0..31)", d[:32], "expected", pc_rows[:32])
print("word p[0][0] lane l = row l&31 word 16h:", d[3072:3072 + 4], "expected", w32[l[:4] & 31, 16 * (l[:4] >> 5)])
seeds = d[64:64 + 1024].view(np.float32).reshape(64, 16)
exp_seed = np.array([[1024 - 0.5 * pc_rows[(g & 3) + 8 * (g >> 2) + 4 * (ll >> 5)] for g in range(16)] for ll in range(64)])
print("seeds ok", np.array_equal(seeds, exp_seed), seeds[0, :4], exp_seed[0, :4])
thb = d[1088:1152].view(np.float32)
print("thb lanes 0..3", thb[:4])
print("wq word lane l:", d[1152:1156], "expected", w32[0:0] if False else qb.view(np.uint32)[l[:4] & 31, 16 * (l[:4] >> 5)])
acc = d[2048:2048 + 1024].view(np.float32).reshape(64, 16)
qbits = np.unpackbits(qb[:32], axis=1).astype(np.int64)
rbits = np.unpackbits(codes[:32], axis=1).astype(np.int64)
dot = rbits @ qbits.T  # [row, query]
exp_acc = np.array([[1024 - 0.5 * pc_rows[(g & 3) + 8 * (g >> 2) + 4 * (ll >> 5)] + dot[(g & 3) + 8 * (g >> 2) + 4 * (ll >> 5), ll & 31]
                     for g in range(16)] for ll in range(64)])
print("acc ok", np.array_equal(acc, exp_acc), acc[0, :4], exp_acc[0, :4], acc[33, :4], exp_acc[33, :4])

# lists after PREFIX + MATRIX (no recheck): counts vs the exact {dist < tau_s} per (query, chunk)
info = np.zeros(12, np.int64)
flags = N.VRQ_SEARCH_PHASE1_ONLY | N.VRQ_SEARCH_SCAN_MFMA
N.check(lib.vrq_scan_plan(n, 1024, nq, K, flags, info.ctypes.data), "plan")
cr, nch, capc, off_cand, off_cnt, off_tau, j = (int(info[i]) for i in (2, 3, 4, 5, 6, 7, 9))
print("plan", info.tolist())
cnt = ws[off_cnt:off_cnt + 4 * nq * nch].view(torch.int32).view(nq, nch).cpu().numpy()
tau_s = ws[off_tau:off_tau + 4 * nq].view(torch.int32).cpu().numpy()
qbits_all = np.unpackbits(qb, axis=1).astype(np.float32)
rbits_all = np.unpackbits(codes, axis=1).astype(np.float32)
Dm = (pcq[:, None] + pc_rows[None, :] - 2 * (qbits_all @ rbits_all.T)).astype(np.int32)
want = np.stack([(Dm[:, c * cr:(c + 1) * cr] < tau_s[:, None]).sum(1) for c in range(nch)], 1)
print("cnt[:4,:6]", cnt[:4, :6])
print("want[:4,:6]", want[:4, :6])
print("equal", np.array_equal(cnt, want), "max cnt", cnt.max(), "max want", want.max(), "capc", capc)

d = ws[:(8192 + 16384 + 1024) * 4].cpu().numpy().view(np.uint32)
rbits1 = np.unpackbits(codes[32:64], axis=1).astype(np.int64)
for qbp in range(15):
    a = d[8192 + qbp * 1024:8192 + qbp * 1024 + 1024].view(np.float32).reshape(64, 16)
    qb_bits = np.unpackbits(qb[qbp * 32:qbp * 32 + 32], axis=1).astype(np.int64)
    dot1 = rbits1 @ qb_bits.T
    exp = np.array([[1024 - 0.5 * pc_rows[32 + (g & 3) + 8 * (g >> 2) + 4 * (ll >> 5)] + dot1[(g & 3) + 8 * (g >> 2) + 4 * (ll >> 5), ll & 31]
                     for g in range(16)] for ll in range(64)])
    print("qblock", qbp, "rb1 acc ok", np.array_equal(a, exp), "nst", d[8192 + 16384 + qbp * 64], a[0, :3], exp[0, :3])
