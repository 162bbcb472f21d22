"""Op-level determinism under memory pressure: every op below runs REPS times on fixed inputs and
each result is compared bit for bit with the first; a second process (`--noise SECONDS`) streams
copies through HBM meanwhile, so memory latencies vary the way they do when another job shares the
device. A kernel whose loads / LDS-DMA are waited for by counting (vmcnt) or ordered by barriers
and gets either wrong shows up here as a run-to-run difference.

    python tools/race_stress.py [REPS] [filter]       (starts its own noise process)
"""
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "comet-pose-estimation_amd")]


def noise(seconds):
    # HBM streaming plus co-resident compute (vendor GEMMs using LDS and every CU): the other
    # process's workgroups then share the CUs with the ops under test and perturb their waves'
    # relative timing, as a second rank on the same device does
    a = torch.empty(512 * 2**20, device="cuda", dtype=torch.float32)  # 2 GiB
    b = torch.empty_like(a)
    x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    y = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    t0 = time.time()
    first = True
    while time.time() - t0 < seconds:
        if first:
            print("noise running", flush=True)
            first = False
        for _ in range(10):
            b.copy_(a)
            z = x @ y
            a.copy_(b)
            z = z @ y
        torch.cuda.synchronize()


def cases():
    from comet_amd import _lib as L, ops
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*shape, dtype=torch.bfloat16, scale=1.0):
        return ((torch.rand(*shape, device="cuda", generator=g) * 2 - 1) * scale).to(dtype)

    out = []
    for (M, N, K, act, odt, res) in [(65536, 1536, 384, L.ACT_GELU, torch.bfloat16, False),
                                     (74368, 2304, 768, L.ACT_NONE, torch.bfloat16, False),
                                     (74368, 768, 3072, L.ACT_NONE, torch.float32, True),
                                     (65536, 1152, 384, L.ACT_NONE, torch.bfloat16, False),
                                     (65536, 384, 384, L.ACT_NONE, torch.bfloat16, False),
                                     (8192, 1536, 384, L.ACT_GELU, torch.bfloat16, False),
                                     (8192, 768, 384, L.ACT_NONE, torch.bfloat16, False),
                                     (65536, 1024, 256, L.ACT_GELU, torch.bfloat16, False)]:
        x, w, b = rnd(M, K), rnd(N, K, scale=0.05), rnd(N, dtype=torch.float32)
        r = rnd(M, N, dtype=odt) if res else None
        aux = torch.empty(M, N, device="cuda", dtype=odt) if act != L.ACT_NONE else None

        def f(x=x, w=w, b=b, r=r, act=act, odt=odt, aux=aux):
            y = ops.linear(x, w, bias=b, act=act, resid=r, out_dtype=odt, aux=aux)
            return (y,) if aux is None else (y, aux)
        out.append((f"linear M{M} N{N} K{K} act{act} {str(odt)[6:]}{' res' if res else ''}", f))
    for (M, N, K, raw, z) in [(65536, 384, 384, True, False), (65536, 384, 1536, False, True),
                              (8192, 384, 1536, False, False), (8192, 384, 384, True, False),
                              (65536, 256, 1024, False, False)]:
        x, w, b = rnd(M, K), rnd(N, K, scale=0.05), rnd(N, dtype=torch.float32)
        r = rnd(M, N, dtype=torch.float32)
        zz = (rnd(N, dtype=torch.float32), rnd(N, dtype=torch.float32), 1e-5) if z else None

        def f(x=x, w=w, b=b, r=r, raw=raw, zz=zz):
            res = ops.linear_rowln(x, w, b, r, raw=raw, y16_eps=1e-6, z=zz)
            return tuple(t for t in (res if isinstance(res, tuple) else (res,)) if torch.is_tensor(t))
        out.append((f"rowln M{M} N{N} K{K} raw{int(raw)} z{int(z)}", f))
    for (B, Lq, Lk, H, D) in [(128, 512, 64, 8, 48), (128, 64, 512, 8, 48), (128, 581, 581, 12, 64),
                              (128, 577, 577, 8, 96), (4096, 16, 16, 8, 48)]:
        q, k, v = rnd(B, Lq, H * D), rnd(B, Lk, H * D), rnd(B, Lk, H * D)

        def f(q=q, k=k, v=v, H=H):
            return ops.attention(q, k, v, H, lse=True)
        out.append((f"attn fwd B{B} Lq{Lq} Lk{Lk} H{H} D{D}", f))
    for (B, L_, H, D) in [(128, 577, 8, 96), (8, 1024, 8, 64)]:
        q, k, v, do = rnd(B, L_, H * D), rnd(B, L_, H * D), rnd(B, L_, H * D), rnd(B, L_, H * D)
        o, lse = ops.attention(q, k, v, H, lse=True)

        def f(q=q, k=k, v=v, o=o, lse=lse, do=do, H=H, D=D):
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            ops.attention_bwd(q, k, v, o, lse, do, H, D ** -0.5, dq, dk, dv)
            return dq, dk, dv
        out.append((f"attn bwd B{B} L{L_} H{H} D{D}", f))
    for (n, h, c, co, k, s) in [(128, 128, 64, 64, 3, 1), (128, 64, 416, 256, 3, 1), (128, 64, 96, 96, 3, 1),
                                (65536, 31, 8, 32, 3, 2), (128, 256, 8, 64, 7, 2)]:
        x, w, b = rnd(n, h, h, c), rnd(co, k * k * c, scale=0.05), rnd(co, dtype=torch.float32)

        def f(x=x, w=w, b=b, k=k, s=s):
            return (ops.conv2d_nhwc(x, w, k, k, s, k // 2, bias=b),)
        out.append((f"conv {k}x{k}s{s} c{c}->{co} {h}^2 n{n}", f))
    return out


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--noise":
        noise(float(sys.argv[2]))
        return
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    nz = subprocess.Popen([sys.executable, __file__, "--noise", "600"], stdout=subprocess.PIPE, text=True)
    try:
        assert nz.stdout.readline().strip() == "noise running", "noise process did not start"
        print("noise process running", flush=True)
        bad = 0
        for name, f in cases():
            if flt not in name:
                continue
            ref = [t.clone() for t in f()]
            torch.cuda.synchronize()
            nd = 0
            worst = 0.0
            for _ in range(reps):
                got = f()
                for a, b in zip(ref, got):
                    if not torch.equal(a, b):
                        nd += 1
                        d = (a.float() - b.float()).abs().max().item()
                        worst = max(worst, d / max(a.float().abs().max().item(), 1e-30))
                        break
            torch.cuda.synchronize()
            bad += nd > 0
            print(f"{'DIFF' if nd else 'ok  '} {nd:3d}/{reps}  worst rel {worst:.2e}  {name}", flush=True)
        print(f"{bad} op(s) not deterministic", flush=True)
    finally:
        nz.kill()
        nz.wait()


if __name__ == "__main__":
    main()
