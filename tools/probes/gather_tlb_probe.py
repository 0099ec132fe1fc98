#!/usr/bin/env python
"""Random 1 KiB row gathers (the config-5 cosine finish's access pattern: ~1.8K candidate rows per query x
1024 queries) from tables of 1M / 4M / 10M int8 rows of 1024 B: is the gather rate set by the table's span
(address translation) rather than by the bytes?  torch.index_select on the GPU, HIP-event timed; one JSON
line per case."""
import json

import torch


def main():
    dev = torch.device("cuda", 0)
    cnt = 1024 * 1784
    big = torch.randint(-127, 128, (10_000_000, 1024), dtype=torch.int8, device=dev)
    for rows in (1_000_000, 4_000_000, 10_000_000):
        tab = big[:rows]
        for order in ("random", "sorted"):
            idx = torch.randint(0, rows, (cnt,), device=dev)
            if order == "sorted":
                idx, _ = torch.sort(idx)
            out = torch.empty((cnt, 1024), dtype=torch.int8, device=dev)
            for _ in range(3):
                torch.index_select(tab, 0, idx, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                torch.index_select(tab, 0, idx, out=out)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            print(json.dumps({"table_rows": rows, "table_gb": rows * 1024 / 1e9, "order": order, "gathers": cnt,
                              "ms": ms, "read_tb_s": cnt * 1024 / (ms * 1e-3) / 1e12}), flush=True)


if __name__ == "__main__":
    main()
