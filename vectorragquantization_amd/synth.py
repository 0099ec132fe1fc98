"""Deterministic synthetic corpora for the BASELINE configs.

Floats: ``F = normalize(C[c_j] + sigma * g_j)`` with 4096 cluster centres
``C ~ N(0, I/d)``, ``sigma = 0.6/sqrt(d)``; ``int8`` = VectorDBInt8Global's
quantiser with limit 0.1 and ``ubinary = packbits(F > 0)`` (the Cohere
relation), both from the gfx950 encode kernel.  Queries: ``normalize(F[j] +
0.3/sqrt(d) * g)`` for random rows j.  Rows are produced in chunks of a fixed
global grid, chunk c seeded ``seed + c``, so any row-sharding over 1/2/4/8 ranks
sees exactly the same rows.  Phase-I-only corpora use uniform random code bytes.
"""
from __future__ import annotations

import math

import torch

from .quant import encode, int8_row_norms

N_CLUSTERS = 4096
SEED = 20250218
QUERY_SEED = 7


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def centres(d: int, device, seed: int = SEED) -> torch.Tensor:
    return torch.randn((N_CLUSTERS, d), generator=_gen(device, seed - 1), device=device) / math.sqrt(d)


def float_rows(c0: int, rows: int, d: int, device, C: torch.Tensor, seed: int = SEED, chunk: int = 0):
    """Float rows of global chunk index ``chunk`` (rows of that chunk only)."""
    g = _gen(device, seed + chunk)
    lab = torch.randint(0, N_CLUSTERS, (rows,), generator=g, device=device)
    F = C[lab] + (0.6 / math.sqrt(d)) * torch.randn((rows, d), generator=g, device=device)
    return F / F.norm(dim=1, keepdim=True)


def chunk_grid(n_total: int, grid_chunks: int = 64):
    """Global chunk size so that shard boundaries of 1/2/4/8 ranks fall on chunk edges."""
    return (n_total + grid_chunks - 1) // grid_chunks


def shard_range(n_total: int, rank: int, world: int, grid_chunks: int = 64):
    cs = chunk_grid(n_total, grid_chunks)
    per = grid_chunks // world
    r0 = min(n_total, rank * per * cs)
    # the last rank takes the grid's remainder when world does not divide grid_chunks
    r1 = n_total if rank == world - 1 else min(n_total, (rank + 1) * per * cs)
    return r0, r1


def make_corpus(n_total: int, d: int = 1024, rank: int = 0, world: int = 1, device="cuda",
                limit: float = 0.1, seed: int = SEED, want_float: bool = False):
    """This rank's shard: dict(codes u8[m,d/8], x8 i8[m,d], norms f64[m], row0, F (optional))."""
    r0, r1 = shard_range(n_total, rank, world)
    cs = chunk_grid(n_total)
    m = r1 - r0
    codes = torch.empty((m, d // 8), dtype=torch.uint8, device=device)
    x8 = torch.empty((m, d), dtype=torch.int8, device=device)
    Fs = [] if want_float else None
    C = centres(d, device, seed)
    step = max(1, min(cs, (1 << 31) // (4 * d)))  # keep each float block < 2 GiB
    for c in range(r0 // cs, (r1 + cs - 1) // cs):
        a, b = c * cs, min((c + 1) * cs, n_total)
        F = float_rows(a, b - a, d, device, C, seed, chunk=c)
        for s in range(0, b - a, step):
            e = encode("cohere", F[s:s + step], limit, device)
            codes[a - r0 + s: a - r0 + s + e["codes"].shape[0]] = e["codes"]
            x8[a - r0 + s: a - r0 + s + e["q"].shape[0]] = e["q"]
        if want_float:
            Fs.append(F)
        del F
    norms = int8_row_norms(x8)
    return {"codes": codes, "x8": x8, "norms": norms, "row0": r0,
            "F": torch.cat(Fs) if want_float else None}


def make_queries(n_total: int, nq: int, d: int = 1024, device="cuda", seed: int = SEED,
                 qseed: int = QUERY_SEED):
    """(qf f32[nq,d], qb u8[nq,d/8], src rows) -- identical on every rank."""
    g = _gen(device, qseed)
    src = torch.randint(0, n_total, (nq,), generator=g, device=device)
    C = centres(d, device, seed)
    cs = chunk_grid(n_total)
    qf = torch.empty((nq, d), dtype=torch.float32, device=device)
    srcl = src.tolist()
    for c in sorted(set(r // cs for r in srcl)):  # regenerate each needed chunk once
        a, b = c * cs, min((c + 1) * cs, n_total)
        F = float_rows(a, b - a, d, device, C, seed, chunk=c)
        for i, r in enumerate(srcl):
            if r // cs == c:
                qf[i] = F[r - a]
        del F
    qf = qf + (0.3 / math.sqrt(d)) * torch.randn((nq, d), generator=g, device=device)
    qf = qf / qf.norm(dim=1, keepdim=True)
    qb = encode("cohere", qf, 0.1, device)["codes"]
    return qf.contiguous(), qb, src


def random_codes(n: int, code_bytes: int = 128, device="cuda", seed: int = SEED):
    """Uniform random code bytes (Phase-I-only roofline corpus), generated in 1 GiB blocks."""
    out = torch.empty((n, code_bytes), dtype=torch.uint8, device=device)
    step = max(1, (1 << 30) // code_bytes)
    for i, s in enumerate(range(0, n, step)):
        g = _gen(device, seed + 1000 + i)
        e = min(n, s + step)
        out[s:e] = torch.randint(0, 256, (e - s, code_bytes), generator=g, device=device, dtype=torch.uint8)
    return out


def flip_queries(codes: torch.Tensor, nq: int, flips=(64, 256), seed: int = QUERY_SEED):
    """Queries = corpus rows with a random number of bit flips in [flips[0], flips[1]]."""
    dev = codes.device
    g = _gen(dev, seed)
    n, cb = codes.shape
    src = torch.randint(0, n, (nq,), generator=g, device=dev)
    q = codes[src].clone()
    mask = torch.zeros((nq, cb * 8), dtype=torch.uint8, device=dev)
    for i in range(nq):
        nf = int(torch.randint(flips[0], flips[1] + 1, (1,), generator=g, device=dev).item())
        mask[i, torch.randperm(cb * 8, generator=g, device=dev)[:nf]] = 1
    w = torch.tensor([128, 64, 32, 16, 8, 4, 2, 1], dtype=torch.int32, device=dev)
    packed = (mask.view(nq, cb, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)
    return q ^ packed, src
