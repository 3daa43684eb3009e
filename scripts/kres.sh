# Register / spill / scratch report of one fast-kernel variant (device-only compile, no GPU).
# usage: bash scripts/kres.sh [pattern] [-DFLAG ...]
#   pattern: mangled-name fragment, default = the headline kernel (f32, Philox, world list, LDS scene)
set -o pipefail
pat=${1:-PhiloxELi0ELb0ELb1ELi0EE}; shift
cd "$(dirname "$0")/../nr-ray-tracer_amd"
out=$(mktemp)
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -fno-fast-math -Wno-unused-function -Icsrc -I../include -x hip \
    --offload-arch=gfx950 -ffp-contract=fast --cuda-device-only -c csrc/kernels_fast.hip -o /dev/null \
    -Rpass-analysis=kernel-resource-usage "$@" > "$out" 2>&1 || { tail -20 "$out"; exit 1; }
grep -A10 "Function Name: .*$pat" "$out" | grep -E "VGPRs:|SGPRs:|Spill|Scratch|Occupancy" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | tr '\n' ' '
echo
rm -f "$out"
