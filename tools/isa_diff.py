"""Per-kernel ISA comparison of two builds of one HIP source (CPU only, no GPU).

Compiles each source for gfx950 with `--cuda-device-only -save-temps` and compares the assembly of
every kernel whose mangled name matches a regex, after normalising what cannot change the executed
instruction stream: block labels, kernel-argument offsets (a grown `Epi` struct shifts them) and
scalar register numbers. Prints, per kernel, the count of differing lines and how many of them are
vector instructions. Used to decide whether a source edit can change a kernel's timing at all
(round 5: the persistent GEMM's A-piece addressing of commit 7a6f28f, profiles/r05_rowln/).

    python tools/isa_diff.py OLD.hip NEW.hip [--match w4] [--show NAME_SUBSTRING]

Each .hip is compiled inside a scratch tree laid out like the repo (csrc/ next to include/), with
the common.hpp / comet_hip.h found next to it or given by --common / --header.
"""
import argparse
import difflib
import os
import re
import shutil
import subprocess
import tempfile

HIPCC = "/opt/rocm/bin/hipcc"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_s(src, common, header, work):
    tree = os.path.join(work, "t")
    os.makedirs(os.path.join(tree, "include"))
    csrc = os.path.join(tree, "x", "csrc")
    os.makedirs(csrc)
    shutil.copy(header, os.path.join(tree, "include", "comet_hip.h"))
    shutil.copy(common, os.path.join(csrc, "common.hpp"))
    shutil.copy(src, os.path.join(csrc, "k.hip"))
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                    "-save-temps=obj", "-c", "k.hip", "-o", "k.o"], cwd=csrc, check=True,
                   stderr=subprocess.DEVNULL)
    return os.path.join(csrc, "k-hip-amdgcn-amd-amdhsa-gfx950.s")


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and line.startswith(".Lfunc_end"):
            out[cur] = body
            cur = None
            continue
        if cur:
            s = line.split(";")[0].strip()
            if not s or (s.startswith(".L") and s.endswith(":")):
                continue
            body.append(re.sub(r"\.LBB\d+_\d+", "L", s))
    return out


def norm(lines):
    o = []
    for x in lines:
        if "kernarg_size" in x or ("sgpr" in x and x.startswith(".")):
            continue
        x = re.sub(r"s\[0:1\], 0x[0-9a-f]+", "s[0:1], OFF", x)
        x = re.sub(r"\bs\[?\d+(:\d+)?\]?", "sX", x)
        o.append(x)
    return o


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("old")
    ap.add_argument("new")
    ap.add_argument("--common-old")
    ap.add_argument("--common-new", default=os.path.join(ROOT, "comet-pose-estimation_amd/csrc/common.hpp"))
    ap.add_argument("--header-old")
    ap.add_argument("--header-new", default=os.path.join(ROOT, "include/comet_hip.h"))
    ap.add_argument("--match", default="w4")
    ap.add_argument("--show")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as w:
        so = compile_s(a.old, a.common_old or a.common_new, a.header_old or a.header_new, os.path.join(w, "o"))
        sn = compile_s(a.new, a.common_new, a.header_new, os.path.join(w, "n"))
        ko, kn = kernels(so), kernels(sn)
    same = 0
    for k in sorted(set(ko) & set(kn)):
        if not re.search(a.match, k):
            continue
        d = [ln for ln in difflib.unified_diff(norm(ko[k]), norm(kn[k]), lineterm="", n=0)
             if ln[:1] in "+-" and ln[:3] not in ("---", "+++")]
        v = [ln for ln in d if "v_" in ln or "vgpr" in ln]
        same += not d
        print(f"{len(d):5d} lines differ ({len(v)} vector)  {k}")
        if a.show and a.show in k:
            print("\n".join(d[:80]))
    print(f"identical after normalisation: {same}; only in old: {len(set(ko) - set(kn))}; "
          f"only in new: {len(set(kn) - set(ko))}")


if __name__ == "__main__":
    main()
