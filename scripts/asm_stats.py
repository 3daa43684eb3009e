"""Static instruction mix of one fast-kernel variant (device-only compile, no GPU).

usage: python scripts/asm_stats.py [mangled-name fragment] [-DFLAG ...]
default fragment: the headline kernel (f32, Philox, world list, LDS scene, KF_FLAT).
Writes the kernel's assembly to /tmp/nrt_kernel.s.
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    args = sys.argv[1:]
    frag = args.pop(0) if args and not args[0].startswith("-") else "PhiloxELi0ELb0ELb1ELi4EE"
    pkg = os.path.join(ROOT, "nr-ray-tracer_amd")
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC", "-fno-fast-math", "-Wno-unused-function", "-Icsrc",
           "-I../include", "-x", "hip", "--offload-arch=gfx950", "-ffp-contract=fast", "-mllvm", "-amdgpu-use-amdgpu-trackers", "--cuda-device-only", "-S",
           "csrc/kernels_fast.hip", "-o", "/tmp/nrt_all.s"] + args
    subprocess.run(cmd, cwd=pkg, check=True, capture_output=True)
    s = open("/tmp/nrt_all.s").read()
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


if __name__ == "__main__":
    main()
