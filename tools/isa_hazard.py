"""Build-time guard for the packed-FP32 operand-select hazard (gfx950, MI355X; round 6).

Measured on the GPU box (profiles/r06_race/README.md, tools/op_repeat.py shflN cases): a packed-FP32
VOP3P instruction -- v_pk_add_f32, v_pk_mul_f32, v_pk_fma_f32 -- whose LOW result reads the HIGH
dword of its second or third source (op_sel bit 1 for src1 / src2) returns wrong values when another
wave on the same SIMD is issuing MFMAs. Reading the first source's high dword (op_sel:[1,..]), the
high result reading a low dword (op_sel_hi), v_pk_mov_b32 and the plain forms are exact under the
same load. The forms arise from hipcc's SLP vectoriser pairing scalar f32 math, which the library
build turns off (-fno-slp-vectorize, Makefile); this script checks the built library for any that
remain and exits non-zero naming the kernels, so a source edit or a compiler update that brings one
back fails the build (__graft_entry__.build(), tests/test_abi.py).

    python tools/isa_hazard.py [library.so]      (default: the product library)

The deliberate instances in comet_shfl_probe (the hazard's own reproducer) are allowed.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
ALLOWED = ("shfl_probe_kernel",)
PK = re.compile(r"\bv_pk_(add|mul|fma)_f32\b")
OPSEL = re.compile(r"op_sel:\[([01](?:,[01])*)\]")


def disassemble(lib):
    """Disassembly of every gfx950 code object in the library (its .hip_fatbin section holds one
    offload bundle per translation unit, back to back)."""
    out = []
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, lib, os.path.join(td, "x.o")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for n, st in enumerate(starts):
            part = os.path.join(td, f"b{n}.bin")
            co = os.path.join(td, f"b{n}.co")
            with open(part, "wb") as f:
                f.write(data[st:starts[n + 1] if n + 1 < len(starts) else len(data)])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + part,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True, capture_output=True)
            out.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout)
    if not out:
        raise RuntimeError(f"isa_hazard: no offload bundle in {lib}")
    return "\n".join(out)


def scan(text):
    """{kernel symbol: [instruction, ...]} of the hazardous forms outside the allowed kernels."""
    bad, kernel = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            kernel = m.group(1)
            continue
        if not PK.search(line):
            continue
        sel = OPSEL.search(line)
        if sel is None:
            continue
        bits = [int(b) for b in sel.group(1).split(",")]
        if any(bits[1:]) and not (kernel and any(a in kernel for a in ALLOWED)):
            bad.setdefault(kernel, []).append(line.strip())
    return bad


def check(lib=None):
    lib = lib or os.path.join(ROOT, "comet-pose-estimation_amd", "libcomet_hip.so")
    return scan(disassemble(lib))


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else None
    bad = check(lib)
    if not bad:
        print("isa_hazard: no packed-FP32 instruction reads a high src1 / src2 dword into its low result")
        return 0
    for k, ins in bad.items():
        print(f"{k}: {len(ins)} instance(s), e.g. {ins[0]}")
    print(f"isa_hazard: {sum(len(v) for v in bad.values())} hazardous instruction(s) in {len(bad)} kernel(s)")
    return 1


if __name__ == "__main__":
    sys.exit(main())
