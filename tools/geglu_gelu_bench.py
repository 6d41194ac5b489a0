"""Routed-GEGLU projection with GELU at the SDXL / SD shapes: the registered-table epilogue (MODE_GEGLU_GT) vs the
fp32 erfc epilogue (table unregistered) -- per-launch device time, warm L2.
usage: python tools/geglu_gelu_bench.py [--iters 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "diffusion-models-moe_amd"), ROOT]

import torch  # noqa: E402

from sdmoe import _lib, ops  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    for M, C in [(16384, 640), (4096, 1280), (65536, 320), (16384, 640 * 2)]:
        F, E = 4 * C, C // 5
        x = torch.randn(M, C, device=dev).half()
        w = (torch.randn(2 * F, C, device=dev) * C ** -0.5).half()
        b = torch.zeros(2 * F, device=dev).half()
        routing = ops.Routing(torch.arange(F) % E, E, E // 5, dev)
        w_il, b_il = ops.interleave_geglu(w, b, routing.perm)
        score = torch.empty(M, E, device=dev).half()
        out = torch.empty(M, F, device=dev).half()
        res = {}
        for name in ("table", "erfc", "relu"):
            act = ops.ACT_RELU if name == "relu" else ops.ACT_GELU
            if name == "table":
                ops.ensure_gelu_table(dev)
            _lib.check(lib.sdmoe_set_gelu_table(ops._GELU_TABLES[0].data_ptr() if name == "table" else None), "tab")
            st = lib.sdmoe_linear_geglu(x.data_ptr(), C, w_il.data_ptr(), C, b_il.data_ptr(), out.data_ptr(), F, M, F,
                                        C, act, score.data_ptr(), E, 20, ops._stream())
            _lib.check(st, "geglu")
            res[name] = timeit(lambda: lib.sdmoe_linear_geglu(x.data_ptr(), C, w_il.data_ptr(), C, b_il.data_ptr(),
                                                              out.data_ptr(), F, M, F, C, act, score.data_ptr(), E, 20,
                                                              ops._stream()), a.iters)
        _lib.check(lib.sdmoe_set_gelu_table(ops._GELU_TABLES[0].data_ptr()), "tab")
        fl = 2.0 * M * 2 * F * C
        print(f"geglu M={M} C={C}: " + "  ".join(f"{k} {v * 1e3:7.1f} us ({fl / v / 1e9:6.0f} TF/s)" for k, v in res.items()))


if __name__ == "__main__":
    main()
