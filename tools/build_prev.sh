#!/bin/bash
# Build the fused kernel of a previous commit (default HEAD) as ablate/librepic_gc_zprev.so, so
# tools/ablate.py times it interleaved with the working tree's build on the same box and clock.
#   bash tools/build_prev.sh [REV]
set -e
REV=${1:-HEAD}
D=repic-copy_amd/csrc
mkdir -p $D/build/prev repic-copy_amd/repic_amd/ablate
for f in rgc_fused.hip rgc_abi.cpp rgc_kernels.hip rgc_kernels.h rgc_device.h pyset.h box_parse.cpp; do
  git show "$REV:$D/$f" > $D/build/prev/$f
done
git show "$REV:include/repic_gc.h" > $D/build/prev/repic_gc.h
H="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function -munsafe-fp-atomics"
cd $D/build/prev
sed -i 's#"../../include/repic_gc.h"#"repic_gc.h"#' *.cpp *.hip *.h
/opt/rocm/bin/hipcc $H -c rgc_fused.hip -o f.o &
/opt/rocm/bin/hipcc $H -c rgc_kernels.hip -o k.o &
g++ -O2 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c rgc_abi.cpp -o a.o &
g++ -O2 -std=c++17 -fPIC -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c box_parse.cpp -o b.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../../repic_amd/ablate/librepic_gc_zprev.so f.o k.o a.o b.o -lpthread
echo "built ablate/librepic_gc_zprev.so from $REV"
