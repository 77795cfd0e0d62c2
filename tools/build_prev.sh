#!/bin/bash
# Build a previous commit's library (default HEAD) as abl/librepic_gc_zprev.so, so
# tools/ablate.py times it interleaved with the working tree's build on the same box and clock.
#   bash tools/build_prev.sh [REV]
set -e
REV=${1:-HEAD}
D=repic-copy_amd/csrc
rm -rf $D/build/prev
mkdir -p $D/build/prev abl
for f in $(git ls-tree --name-only "$REV" $D/ | xargs -n1 basename); do
  git show "$REV:$D/$f" > $D/build/prev/$f
done
git show "$REV:include/repic_gc.h" > $D/build/prev/repic_gc.h
H="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function -munsafe-fp-atomics"
cd $D/build/prev
sed -i 's#"../../include/repic_gc.h"#"repic_gc.h"#' *.cpp *.hip *.h
objs=""
for f in *.hip; do /opt/rocm/bin/hipcc $H -c $f -o ${f%.hip}.o & objs="$objs ${f%.hip}.o"; done
for f in *.cpp; do g++ -O2 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $f -o ${f%.cpp}.o & objs="$objs ${f%.cpp}.o"; done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../../../abl/librepic_gc_zprev.so $objs -lpthread
echo "built abl/librepic_gc_zprev.so from $REV"
