"""Run tools/probes/mmr_fold.hip: the lower bound of an MMR layout that keeps
candidate rows out of the register file.
1M users x C = 1000 candidates (random rows of a 10M x 128 bf16 table, as
config 5's lists) x 8 fold passes per user (the product's batches per user
on real top-1000 lists), at 2 / 4 / 8 users in flight per CU. Prints one JSON
line: ms per 1M users and the row bytes streamed.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probes/mmr_fold.hip -o tools/probes/libmmr_fold.so
    python tools/probes/mmr_fold.py
"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libmmr_fold.so"))
    lib.probe_mmr_fold.restype = ctypes.c_int
    lib.probe_mmr_fold.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    n_items, d, C, n_users, batches = 10_000_000, 128, 1000, 1_000_000, 8
    g = torch.Generator(device=dev).manual_seed(11)
    E = (torch.randn(n_items, d, device=dev, generator=g) / d ** 0.5).to(torch.bfloat16)
    cand = torch.randint(0, n_items, (n_users, C), device=dev, generator=g, dtype=torch.int32)
    out = torch.empty(n_users, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    res = {"users": n_users, "candidates": C, "d": d, "batches": batches,
           "row_bytes": n_users * batches * C * d * 2, "ms": {}}
    for per_cu in (2, 4, 8):
        grid = cus * per_cu
        times = []
        for rep in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lib.probe_mmr_fold(E.data_ptr(), n_items, cand.data_ptr(), C, n_users, batches,
                                      grid, out.data_ptr(), stream) == 0
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        res["ms"][per_cu] = min(times)
        print(f"users/CU {per_cu}: {times}", flush=True)
    best = min(res["ms"].values())
    res["best_ms"] = best
    res["row_tb_per_s"] = res["row_bytes"] / (best * 1e-3) / 1e12
    print(json.dumps(res))


if __name__ == "__main__":
    main()
