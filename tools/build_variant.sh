#!/bin/bash
# tools/build_variant.sh NAME [extra hipcc flags...] -- builds polymutt_amd/lib_exp/NAME.so: the engine with
# experimental compile-time switches, linked with the regular host objects (select it with POLYMUTT_LIB).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
mkdir -p "$R/polymutt_amd/lib_exp" /tmp/pm_variants
make -s -C "$R/polymutt_amd" lib/libpolymutt.so
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -w "$@" \
  -c -x hip "$R/polymutt_amd/csrc/engine.hip" -o /tmp/pm_variants/$NAME.o
objs=$(ls "$R"/polymutt_amd/build/*.o | grep -v engine.o)
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$R/polymutt_amd/lib_exp/$NAME.so" /tmp/pm_variants/$NAME.o $objs -lz -lhiprtc -pthread
echo "built polymutt_amd/lib_exp/$NAME.so"
