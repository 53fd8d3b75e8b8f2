#!/usr/bin/env python3
"""Development tool: a library variant of dq_kernels.hip with textual
ablations (the product source is not touched): copies csrc/ to a temp dir,
applies the named patches, builds tools/bin/NAME.so against the tree's other
objects.   python3 tools/psvar_patch.py NAME PATCH [PATCH...]
Patches: acc0 -- partsplit without the children's per-(tile, wave) counts;
sum0 -- partsplit without the children's split sums."""
import os
import shutil
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCHES = {
    "acc0": [("    chunk_sweep(cx, oc, g.cbo + g.po, om, xm, xc);\n    chunk_sweep(cy, nc, g.cbn + g.pn - kPnOff, nm, ym, yc);",
              "    (void)oc; (void)nc;"),
             ("  chunk_finish(cx);\n  chunk_finish(cy);\n}", "}")],
    "sum0": [("    if (kSums) {\n      add_sums_bytes(sw, xm, xc, so);", "    if (false) {\n      add_sums_bytes(sw, xm, xc, so);")],
}


def main():
    name, pats = sys.argv[1], sys.argv[2:]
    tmp = tempfile.mkdtemp()
    try:
        src = os.path.join(tmp, "csrc")
        shutil.copytree(os.path.join(R, "clusteringsegmentation-1_amd", "csrc"), src)
        p = os.path.join(src, "dq_kernels.hip")
        s = open(p).read()
        for pat in pats:
            for a, b in PATCHES[pat]:
                assert s.count(a) == 1, (pat, a)
                s = s.replace(a, b)
        open(p, "w").write(s)
        B = os.path.join(R, "clusteringsegmentation-1_amd", "build")
        obj = os.path.join(tmp, "k.o")
        os.makedirs(os.path.join(R, "tools", "bin"), exist_ok=True)
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                               "-ffp-contract=off", "-fno-fast-math", "-c", "-o", obj, p])
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o",
                               os.path.join(R, "tools", "bin", name + ".so"), obj] +
                              [os.path.join(B, o) for o in ("dq_weighted.o", "dq_engine.o", "dq_abi.o", "build_id.o")] +
                              ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
        print("built tools/bin/%s.so" % name)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()
