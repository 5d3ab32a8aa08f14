"""Run tools/probes/mfma_shape.hip: TFLOP/s of bare 32x32x16 and 16x16x32 bf16
MFMA loops on random operands, one 512-thread workgroup per CU, each shape
timed on one ~2.7-ms launch per round, three alternating rounds. Prints one
JSON line.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probes/mfma_shape.hip -o tools/probes/libmfma_shape.so
    python tools/probes/mfma_shape.py
"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libmfma_shape.so"))
    lib.probe_mfma.restype = ctypes.c_int
    lib.probe_mfma.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    g = torch.Generator(device=dev).manual_seed(7)
    src = torch.randn(1 << 22, device=dev, generator=g).to(torch.bfloat16)  # 8 MiB random bf16
    out = torch.empty(cus * 512, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    iters = 20000
    flops = cus * 8 * 4 * (2 * 32 * 32 * 16) * iters  # 8 waves x 4 x 32x32x16 MACs x 2 per iteration
    res = {32: [], 16: []}
    for rnd in range(3):
        for shape in (32, 16):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            assert lib.probe_mfma(shape, src.data_ptr(), cus, iters, out.data_ptr(), stream) == 0
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            res[shape].append(flops / (ms * 1e-3) / 1e12)
    print(json.dumps({"cus": cus, "iters": iters,
                      "tflops_32x32x16": res[32], "tflops_16x16x32": res[16],
                      "ratio_16_over_32": [b / a for a, b in zip(res[32], res[16])]}), flush=True)


if __name__ == "__main__":
    main()
