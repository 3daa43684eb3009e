"""Static instruction mix and register use of one render-kernel variant (device-only compile, no GPU).

usage: python scripts/asm_stats.py [--exact] [mangled-name fragment] [-DFLAG ...]
       python scripts/asm_stats.py --targs "float, nrt::dev::Philox, -1, false, false, 4, nrt::dev::BvhSig<4, false>"
default fragment: the headline kernel (f32, Philox, world list, LDS scene, KF_FLAT) of kernels_fast.hip.
--targs: the template arguments of a scene-specialised kernel (jit.hip builds them with hiprtc; the
bench line's `pmc.kernel` names them), instantiated here with hipcc and the JIT's flags.
Writes the kernel's assembly to /tmp/nrt_kernel.s and prints VGPR / SGPR / spill / occupancy figures.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["-std=c++17", "-O3", "-fPIC", "-fno-fast-math", "-Wno-unused-function", "-x", "hip", "--offload-arch=gfx950",
         os.environ.get("CONTRACT", "-ffp-contract=on"), "-mllvm", "-amdgpu-use-amdgpu-trackers", "--cuda-device-only", "-S",
         "-Rpass-analysis=kernel-resource-usage"]


def main():
    args = sys.argv[1:]
    pkg = os.path.join(ROOT, "nr-ray-tracer_amd")
    inc = ["-I" + os.path.join(pkg, "csrc"), "-I" + os.path.join(ROOT, "include")]
    td = tempfile.mkdtemp()
    flags = list(FLAGS)
    exact = bool(args) and args[0] == "--exact"
    if exact:  # the exact kernels' contraction (kernels_exact.hip: none)
        flags = [f if f != os.environ.get("CONTRACT", "-ffp-contract=on") else "-ffp-contract=off" for f in flags]
        flags = [f for f in flags if f not in ("-mllvm", "-amdgpu-use-amdgpu-trackers")]
        args = args[1:]
    if args and args[0] == "--targs":
        targs = args[1]
        args = args[2:]
        src = os.path.join(td, "jit_variant.hip")
        with open(src, "w") as fh:
            fh.write('#include "kernel.hpp"\n'
                     f"template __global__ void nrt::dev::render_kernel<{targs}>(const nrt::RenderParams, "
                     f"const nrt::DSceneView<{targs.split(',')[0].strip()}>);\n")
        frag = ""
    else:
        frag = args.pop(0) if args and not args[0].startswith("-") else "PhiloxELi0ELb0ELb1ELi4EE"
        src = os.path.join(pkg, "csrc", "kernels_exact.hip" if exact else "kernels_fast.hip")
    out = os.path.join(td, "all.s")
    r = subprocess.run(["/opt/rocm/bin/hipcc", *flags, *inc, src, "-o", out, *args], cwd=pkg, capture_output=True,
                       text=True)
    if r.returncode != 0:
        sys.exit(r.stderr[-3000:])
    s = open(out).read()
    m = re.search(r"^(_ZN3nrt3dev13render_kernel\S*%s\S*):" % re.escape(frag), s, re.M)
    if not m:
        sys.exit(f"no kernel matching {frag}")
    i = m.start()
    body = s[i:s.index(".Lfunc_end", i)]
    open("/tmp/nrt_kernel.s", "w").write(body)
    ins = [l.strip() for l in body.split("\n")]
    ins = [l for l in ins if l and not l.startswith((".", ";")) and not l.endswith(":")]
    c = collections.Counter(l.split()[0] for l in ins)
    valu = sum(n for k, n in c.items() if k.startswith("v_"))
    salu = sum(n for k, n in c.items() if k.startswith("s_"))
    print(f"{m.group(1)[:90]}\ninstructions {len(ins)}  valu {valu}  salu/branch {salu}")
    print("  ".join(f"{k} {n}" for k, n in c.most_common(30)))
    # kernel-resource-usage remarks of this kernel (VGPRs, SGPRs, spills, scratch, occupancy)
    lines = r.stderr.split("\n")
    for k, line in enumerate(lines):
        if "Function Name:" in line and m.group(1) in line:
            res = []
            for l2 in lines[k + 1:k + 14]:
                if re.search(r"VGPRs:|AGPRs:|SGPRs:|Spill|ScratchSize|Occupancy|LDS Size", l2):
                    res.append(re.sub(r".*remark: *", "", l2).split(" [-Rpass")[0].strip())
            print("  ".join(res))
            break


if __name__ == "__main__":
    main()
