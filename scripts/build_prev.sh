# Build libnrt.so from the last commit (or the revision given as $1)'s sources into nr-ray-tracer_amd/ab/prev (A/B baseline for
# scripts/ab_configs.py --arm prev=nr-ray-tracer_amd/ab/prev/libnrt.so).
set -e
cd "$(dirname "$0")/../nr-ray-tracer_amd/ab"
rm -rf prevpkg prev prev_obj
mkdir -p prevpkg/csrc
cp ../Makefile prevpkg/
rev=${1:-HEAD}
for f in $(git ls-files ../csrc); do git show $rev:nr-ray-tracer_amd/csrc/$(basename $f) > prevpkg/csrc/$(basename $f) 2>/dev/null || rm -f prevpkg/csrc/$(basename $f); done
ln -sfn ../../include include
make -C prevpkg -j8 OUT=../prev OBJ=../prev_obj ../prev/libnrt.so > /dev/null
ls -la prev/libnrt.so
