#!/bin/bash
# tools/build_variant.sh NAME [extra hipcc flags...] -- builds polymutt_amd/lib_exp/NAME.so: the engine with
# experimental compile-time switches, linked with the regular host objects (select it with POLYMUTT_LIB).
# Both device halves get the flags: engine.hip and the eight k_brent parts (brent_inst.hip, PM_BRENT_PART 0-7), so a
# switch in engine_dev.h reaches every kernel and DevArgs stays one layout across the objects.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
D=/tmp/pm_variants/$NAME
mkdir -p "$R/polymutt_amd/lib_exp" "$D"
make -s -C "$R/polymutt_amd" lib/libpolymutt.so
F=(-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics -w "$@")
/opt/rocm/bin/hipcc "${F[@]}" -c -x hip "$R/polymutt_amd/csrc/engine.hip" -o "$D/engine.o" &
for k in 0 1 2 3 4 5 6 7; do
  /opt/rocm/bin/hipcc "${F[@]}" -DPM_BRENT_PART=$k -c -x hip "$R/polymutt_amd/csrc/brent_inst.hip" -o "$D/brent_inst_$k.o" &
done
wait
for k in 0 1 2 3 4 5 6 7; do [ -s "$D/brent_inst_$k.o" ] || { echo "part $k failed" >&2; exit 1; }; done
[ -s "$D/engine.o" ] || { echo "engine.o failed" >&2; exit 1; }
objs=$(ls "$R"/polymutt_amd/build/*.o | grep -v -e '/engine.o$' -e '/brent_inst_' -e '/jit_check.o$')
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o "$R/polymutt_amd/lib_exp/$NAME.so" "$D"/engine.o "$D"/brent_inst_*.o $objs -lz -lhiprtc -pthread
echo "built polymutt_amd/lib_exp/$NAME.so"
