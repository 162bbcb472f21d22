"""Map rocprofv3 kernel names (mangled or demangled) to the kernel-instance names bench.py's
live profiler uses (comet_amd/ops.py _plan_name / attention):

    big::gemm_big_kernel<__bf16, 256, 0, 0, false, 0>  ->  comet_gemm|big256.L00.bf16
    attn_fwd_kernel<__bf16, 64>                          ->  comet_attention_fwd|tile.bf16.D64

Non-comet kernels (torch) map to None.
"""
import re

_MANGLED_TYPES = {"DF16b": "bf16", "f": "f32", "b": "bool", "i": "int"}


def _parse_mangled(name):
    """_ZN5comet12_GLOBAL__N_13big15gemm_big_kernelIDF16bLi256ELi0E...EE... -> (base, [args])"""
    if not name.startswith("_ZN"):
        return None
    i, idents = 3, []
    while i < len(name) and name[i].isdigit():
        j = i
        while name[j].isdigit():
            j += 1
        n = int(name[i:j])
        idents.append(name[j:j + n])
        i = j + n
    if i >= len(name) or name[i] != "I" or not idents:
        return None
    i += 1
    args = []
    while i < len(name) and name[i] != "E":
        if name.startswith("DF16b", i):
            args.append("bf16")
            i += 5
        elif name[i] == "L":  # literal: L<type><value>E
            m = re.match(r"L([a-z])(n?\d+)E", name[i:])
            if not m:
                return None
            v = m.group(2).replace("n", "-")
            args.append(("true" if v == "1" else "false") if m.group(1) == "b" else v)
            i += m.end()
        elif name[i] in _MANGLED_TYPES:
            args.append(_MANGLED_TYPES[name[i]])
            i += 1
        else:
            return None
    return idents[-1], args


def _parse_demangled(name):
    m = re.search(r"(\w+)<([^()]*)>\(", name)
    if not m:
        m2 = re.search(r"(\w+)\(", name)
        return (m2.group(1), []) if m2 else None
    args = [a.strip() for a in m.group(2).split(",")]
    args = ["bf16" if a in ("__bf16", "bool _Accum") else ("f32" if a == "float" else a) for a in args]
    return m.group(1), args


def parse(name):
    return _parse_mangled(name) or _parse_demangled(name)


def instance(name):
    """comet kernel-instance name, or None for a kernel outside libcomet_hip."""
    if "comet" not in name:
        return None
    p = parse(name)
    if p is None:
        return None
    base, a = p
    try:
        if base == "gemm_big_kernel":
            tc, bn, la, lb, split = a[0], a[1], a[2], a[3], a[4]
            return f"comet_gemm|big{bn}.L{la}{lb}.{'split' if split == 'true' else tc}"
        if base == "gemm_w4_kernel":  # <TC, ACT, HASR, NW, TBM, TBN, LN, PING>
            # index from the end: the demangler sometimes splits an enum ACT argument in two
            if a[-2] == "true":
                return "comet_gemm_rowln"
            return f"comet_gemm|pp{a[-4]}x{a[-3]}.L00.{a[0]}"
        if base == "gemm_bf16_kernel":
            tc, la, lb, split, conv = a[0], a[1], a[2], a[5], a[6]
            if conv == "true":
                return f"comet_conv2d_nhwc|tile128.{'split' if split == 'true' else tc}"
            return f"comet_gemm|tile128.L{la}{lb}.bf16.{'split' if split == 'true' else tc}"
        if base == "gemm_f32_kernel":
            return "comet_gemm|tile128.f32"
        if base == "gemm_skinny_kernel":
            return "comet_gemm|skinny"
        if base == "conv_skinny_kernel":
            return "comet_conv2d_nhwc|skinny"
        if base == "attn_fwd_kernel":
            return f"comet_attention_fwd|tile.{a[0]}.D{a[1]}"
        if base == "attn_fwd_bf16_kernel":
            return f"comet_attention_fwd|tile.bf16.D{a[0]}"
        if base == "attn_small_kernel":
            return f"comet_attention_fwd|small.bf16.D{a[0]}"
        if base in ("attn_bwd_dkdv2_kernel", "attn_bwd_dq2_kernel", "attn_delta_bf16_kernel"):
            return f"comet_attention_bwd|{base}"
    except IndexError:
        return None
    return base


if __name__ == "__main__":
    import sys
    for n in sys.argv[1:]:
        print(instance(n), parse(n))
