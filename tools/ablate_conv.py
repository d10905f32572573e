"""Build ablated variants of the conv3x3 kernel (each with one piece of work removed) into
build/abl/lib<variant>.so, for tools/ab_conv.py-style timing against the full kernel:
what each piece costs is what its removal buys.  Variants:
  noload  : no global loads of the staged chunk (registers hold a lane-dependent value)
  nostage : no staging at all (no loads, no LDS stores; LDS holds stale data)
  nowload : no weight loads in the K loop (prologue weights reused)
  noepi   : epilogue reduced to keeping the accumulators alive
Outputs differ from the full kernel by construction; only the timings mean anything."""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "data_diet_distributed_amd", "csrc")
OUT = os.path.join(ROOT, "build", "abl")

EDITS = {
    "full": [],
    "noload": [(r"ra\[k\] = \*reinterpret_cast<const float4\*>\(x \+ \(\(size_t\)bc \* cin \+ cgc\) \* HW \+ irc \* W \+\s*x4 \* 4\);",
                "ra[k] = make_float4((float)q, (float)c0, 1.f, 2.f);")],
    "nostage": [(r"      load_chunk\(Tp, kn \* CC\);\n", ""), (r"      store_chunk\(cur \^ 1\);\n", "")],
    "nowload": [(r"      if \(wload\) load_w_taps\(Tp\.ob32, kn, \d, 3\);\n", "")],
    "noepi": [(r"    epilogue\(T, tile, \(g - 1\) & 1\);\n",
               "    { float z = 0.f;\n      for (int a_ = 0; a_ < NA; ++a_) for (int n_ = 0; n_ < NT; ++n_)"
               " for (int r_ = 0; r_ < 16; ++r_) z += acc[a_][n_][r_];\n"
               "      if (z == 1.2345f) A.y[tid] = z; }\n")],
}
# down_fwd variants (dd_down.hip): what the epilogue / staging cost the downsampling head
DOWN_EDITS = {
    "down_noepi": [(r"      epilogue\(T, acc\[a\], A\.main, T\.o_w \+ 32 \* a, red_buf\);\n"
                    r"      if constexpr \(SC\) epilogue\(T, acc_s\[a\], A\.sc, T\.o_w \+ 32 \* a, red_buf\);\n",
                    "      { float z = 0.f; for (int r_ = 0; r_ < 16; ++r_) z += acc[a][r_] + acc_s[a][r_];\n"
                    "        if (z == 1.2345f) A.main.y[tid] = z; }\n")],
    "down_nostage": [(r"      load_chunk\(Tp, kn \* CC\);\n", ""),
                     (r"      store_chunk\(cur \^ 1\);\n", "")],
}
EDITS.update(DOWN_EDITS)
# conv1x1_kernel variants (dd_conv1x1.hip)
C1_EDITS = {
    "c1_noload": [(r"ra\[k\] = \*reinterpret_cast<const float4\*>\(src\);",
                   "ra[k] = make_float4((float)k, (float)tid, 1.f, 2.f);")],
    "c1_nostage": [(r"        load_chunk\(T, kc \+ 1\);\n", ""),
                   (r"        store_chunk\(T, kc \+ 1, cur \^ 1\);\n", "")],
    "c1_noepi": [(r"    epilogue\(T\);\n",
                  "    { float z = 0.f;\n      for (int a_ = 0; a_ < NA; ++a_) for (int n_ = 0; n_ < NT; ++n_)"
                  " for (int r_ = 0; r_ < 16; ++r_) z += acc[a_][n_][r_];\n"
                  "      if (z == 1.2345f) A.y[tid] = z; }\n")],
}
EDITS.update(C1_EDITS)


def build(variant):
    d = os.path.join(OUT, variant)
    os.makedirs(os.path.join(d, "data_diet_distributed_amd", "csrc"), exist_ok=True)
    os.makedirs(os.path.join(d, "include"), exist_ok=True)
    shutil.copy(os.path.join(ROOT, "include", "dd_capi.h"), os.path.join(d, "include"))
    for h in ("dd_common.h", "dd_mfma.h"):
        shutil.copy(os.path.join(SRC, h), os.path.join(d, "data_diet_distributed_amd", "csrc"))
    name = ("dd_down" if variant.startswith("down_") else
            "dd_conv1x1" if variant.startswith("c1_") else "dd_conv")
    s = open(os.path.join(SRC, name + ".hip")).read()
    for pat, rep in EDITS[variant]:
        s, n = re.subn(pat, rep, s)
        assert n > 0, (variant, pat)
    src = os.path.join(d, "data_diet_distributed_amd", "csrc", name + ".hip")
    open(src, "w").write(s)
    obj = os.path.join(d, name + ".o")
    flags = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", src, "-o", obj],
                          stderr=subprocess.DEVNULL)
    others = [os.path.join(OUT, "obj", f) for f in sorted(os.listdir(os.path.join(OUT, "obj")))
              if f != name + ".o"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-shared", "-o",
                           os.path.join(OUT, f"lib{variant}.so"), obj, *others])


if __name__ == "__main__":
    for v in sys.argv[1:] or EDITS:
        build(v)
        print("built", v, flush=True)
