#!/usr/bin/env python3
"""Host -> device copy rates on this box (the upload half of the processing time).

Pinned 32 MiB chunks on one stream (gx_graph_create's staging size), the same on two streams,
one large pinned copy, and a pageable copy.  Prints one JSON line.

    python tools/h2d_probe.py [--mib 2560]
"""
import argparse
import json
import time

import torch


def rate(fn, nbytes, reps=3):
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = max(best, nbytes / (time.perf_counter() - t) / 1e9)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=2560)
    args = ap.parse_args()
    total = args.mib << 20
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    out = {}
    for chunk_mib in (8, 32, 128):
        chunk = chunk_mib << 20
        bufs = [torch.empty(chunk, dtype=torch.uint8).pin_memory() for _ in range(2)]
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]

        def one():
            s = streams[0]
            with torch.cuda.stream(s):
                for i, off in enumerate(range(0, total, chunk)):
                    dev[off:off + chunk].copy_(bufs[i & 1], non_blocking=True)

        def two():
            for i, off in enumerate(range(0, total, chunk)):
                with torch.cuda.stream(streams[i & 1]):
                    dev[off:off + chunk].copy_(bufs[i & 1], non_blocking=True)
        out[f"pinned_{chunk_mib}mib_1stream_gbs"] = round(rate(one, total), 2)
        out[f"pinned_{chunk_mib}mib_2streams_gbs"] = round(rate(two, total), 2)
    big = torch.empty(total, dtype=torch.uint8).pin_memory()
    out["pinned_one_copy_gbs"] = round(rate(lambda: dev.copy_(big, non_blocking=True), total), 2)
    del big
    pg = torch.ones(total, dtype=torch.uint8)
    out["pageable_one_copy_gbs"] = round(rate(lambda: dev.copy_(pg), total), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
