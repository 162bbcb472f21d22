"""Does a kernel leave LDS writes in flight when its workgroups end? (round 6 check)

Stream 1 runs the persistent GEMM on shapes whose epilogue issues no load (bf16 output, no bias, no
residual: the tracker's q / kv projections), so its trailing k-tile re-loads were drained only by
the exit wait; stream 2 runs comet_lds_probe -- workgroups that own a CU's whole LDS, fill it with a
pattern, sleep and count the words that changed. Probe workgroups are placed on a CU as GEMM
workgroups leave it, so LDS-DMA pieces still in flight at s_endpgm would land in the probe's LDS and
be counted. Measured (profiles/r06_race): 0 words with and without the exit wait -- this was not
the cause of round 5's two-process variation (that is the packed-FP32 operand-select hazard,
tools/isa_hazard.py).

    python tools/lds_race.py [iters]          (COMET_HIP_LIB selects the library under test)

Prints one line per shape: probe words overwritten (0 = clean).
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "comet-pose-estimation_amd")]

# (M, N, K): 128 x 384 tiles (N = 384), 256 x 256 lock-step (K < 768), 256 x 256 ping-pong (K 768)
SHAPES = [(65536, 384, 384), (65536, 1536, 384), (74368, 2304, 768)]


def run(iters=40, shapes=SHAPES, groups=1024, rounds=2, spin=2):
    from comet_amd import _lib as L
    from comet_amd import ops
    lib = L.load()
    torch.manual_seed(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}
    for (M, N, K) in shapes:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        bad = torch.zeros(1, device="cuda", dtype=torch.int32)
        torch.cuda.synchronize()
        for _ in range(iters):
            with torch.cuda.stream(s1):
                ops.linear(x, w)
            with torch.cuda.stream(s2):
                L.check(lib.comet_lds_probe(groups, rounds, spin, ctypes.c_void_p(bad.data_ptr()), ops.stream()),
                        "comet_lds_probe")
        torch.cuda.synchronize()
        out[(M, N, K)] = int(bad.item())
        del x, w
    return out


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    from comet_amd import _lib as L
    print(f"library {L.LIB_PATH}", flush=True)
    for shape, n in run(iters).items():
        print(f"M {shape[0]} N {shape[1]} K {shape[2]}: {n} probe LDS words overwritten over {iters} iterations", flush=True)


if __name__ == "__main__":
    main()
