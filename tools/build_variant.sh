#!/bin/bash
# Build an experimental libipmc.so that differs from the product build in one
# translation unit's flags (layout / occupancy experiments), reusing the other
# objects of build/ipmc.  Select it at run time with IPMC_LIB_PATH.
#   tools/build_variant.sh <name> <unit.hip> <extra hipcc flags...>
#   -> ip_mcmc_amd/lib/variants/<name>/libipmc.so
set -e
name=$1; unit=$2; shift 2
cd "$(dirname "$0")/../ip_mcmc_amd/csrc"
out=../lib/variants/$name
mkdir -p "$out" ../../build/variants/$name
obj=../../build/variants/$name/${unit%.hip}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
  -Wall -Wno-unused-function "$@" -c "$unit" -o "$obj"
objs=$obj
for o in ../../build/ipmc/*.o; do
  [ "$(basename "$o")" = "$(basename "$obj")" ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libipmc.so" $objs
echo "$out/libipmc.so"
