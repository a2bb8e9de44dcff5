#!/usr/bin/env bash
# A/B build of libsbr with extra -D flags (every source):
#   tools/build_variant.sh NAME "-DFOO -DBAR=2"  ->  replication-social-bank-runs_amd/lib_var/NAME/libsbr.so
# (run bench.py / tests against it with SBR_LIB=<that path>)
set -eu
cd "$(dirname "$0")/../replication-social-bank-runs_amd"
make -s all
name=$1; defs=${2:-}
mkdir -p build_var/$name lib_var/$name
objs=""
for f in sbr_baseline sbr_hetero sbr_social sbr_capi sbr_multi; do
  if [ -n "$defs" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
      -fno-gpu-flush-denormals-to-zero -Wno-unused-function $defs -c -o build_var/$name/$f.o csrc/$f.hip &
    objs="$objs build_var/$name/$f.o"
  else
    objs="$objs build/$f.o"
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib_var/$name/libsbr.so $objs -ldl -lpthread
echo "lib_var/$name/libsbr.so"
