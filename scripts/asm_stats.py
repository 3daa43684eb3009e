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
        frag = args.pop(0) if args and not args[0].startswith("-") else "PhiloxELi0ELb0ELb1ELi4ENS0_5NoSig"
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
    loop_classes(body)
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


# rocprofv3's SQ_INSTS_VALU_* classes (the PMC passes' valu_mix), by opcode; the rest is "OTHER"
CLASSES = [("TRANS_F32", r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_(iflag_)?f32"), ("TRANS_F64", r"^v_(rcp|rsq|sqrt)_f64"),
           ("FMA_F64", r"^v_(fma|fmac)_f64|^v_div_fmas_f64"), ("MUL_F64", r"^v_mul_f64"), ("ADD_F64", r"^v_add_f64"),
           ("FMA_F32", r"^v_(fma|fmac|fmaak|fmamk|mad|mac|pk_fma|fma_mix)\w*_f32"), ("MUL_F32", r"^v_(pk_)?mul_f32"),
           ("ADD_F32", r"^v_(pk_)?(add|sub|subrev)_f32"), ("CVT", r"^v_cvt_"), ("INT64", r"^v_(mad_u64_u32|lshl_add_u64|\w+_u64|\w+_i64)"),
           ("INT32", r"^v_(add|sub|subrev|mul_lo|mul_hi|mad_u32|mad_i32|lshl|lshr|ashr|and|or|xor|not|bfe|bfi|alignbit|"
                     r"bitop3|perm|add3|lshl_add|lshl_or|and_or|or3|xad|min_u32|max_u32|min_i32|max_i32|bcnt|mbcnt)\w*")]


def loop_classes(body):
    """Static VALU mix of the kernel's outermost loop (first `Loop Header: Depth=1` block to its last
    back-edge), in rocprofv3's SQ_INSTS_VALU_* classes, with OTHER broken down by opcode: what the
    profile's valu_mix OTHER share is made of (compares, selects, moves, min/max, lane moves)."""
    lines = body.split("\n")
    best = None
    for head, l in enumerate(lines):  # the largest outermost loop (the staging loops before it are small)
        if "Loop Header: Depth=1" not in l:
            continue
        label = l.split(":")[0].strip()
        tail = max((i for i, x in enumerate(lines) if re.search(r"s_(c)?branch\w*\s+" + re.escape(label) + r"\b", x)),
                   default=None)
        if tail is not None and tail > head and (best is None or tail - head > best[1] - best[0]):
            best = (head, tail)
    if best is None:
        return
    head, tail = best
    ops = [l.strip().split()[0] for l in lines[head:tail + 1]
           if l.strip() and not l.strip().startswith((".", ";")) and not l.strip().endswith(":")]
    valu = [o for o in ops if o.startswith("v_")]
    cls = collections.Counter()
    other = collections.Counter()
    for o in valu:
        k = next((name for name, rx in CLASSES if re.match(rx, o)), "OTHER")
        cls[k] += 1
        if k == "OTHER":
            other[re.sub(r"_e(32|64)$", "", o)] += 1
    print(f"outer loop (lines {head}-{tail}): {len(ops)} instructions, {len(valu)} VALU")
    print("  classes: " + "  ".join(f"{k} {n} ({n / len(valu):.0%})" for k, n in cls.most_common()))
    print("  OTHER:   " + "  ".join(f"{k} {n}" for k, n in other.most_common(16)))


if __name__ == "__main__":
    main()
