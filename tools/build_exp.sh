#!/bin/bash
# Measurement-only build of libpbnsim with extra -D flags (e.g. -DPBN_PHILOX_ROUNDS=2 to size the
# RNG's share of a kernel) and/or experiment patches from tools/patches/ applied to a copy of csrc/
# (the dropped variants measured in earlier rounds live there, not in the product source).
# Usage: tools/build_exp.sh TAG [-p tools/patches/X.patch]... [-DFLAG]...
# Output: build_exp/<tag>/libpbnsim.so; use with PBNSIM_LIB=... Never used by the product, tests or bench.py.
set -e
tag=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
out=$R/build_exp/$tag
rm -rf $out
mkdir -p $out/src
cp -r $R/gym-pbn-stac_amd/csrc $out/src/csrc
mkdir -p $out/include && cp $R/include/*.h $out/include/
flags=()
while [ $# -gt 0 ]; do
  if [ "$1" = "-p" ]; then
    (cd $out/src && patch -p1 --no-backup-if-mismatch < "$R/$2" > /dev/null) || { echo "patch $2 failed"; exit 1; }
    shift 2
  else
    flags+=("$1"); shift
  fi
done
cd $out/src
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -mcode-object-version=5 -Wno-pass-failed -I$out/include ${flags[*]}"
for k in pbn_kernels pbn_mt pbn_ssd pbn_sync; do /opt/rocm/bin/hipcc $F -c -o $out/$k.o csrc/$k.hip & done
g++ -O2 -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$out/include ${flags[*]} -c -o $out/pbn_abi.o csrc/pbn_abi.cpp
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libpbnsim.so $out/*.o -L/opt/rocm/lib -lamdhip64
echo built $out/libpbnsim.so
