#!/bin/bash
# Experiment library: the product objects with one of them rebuilt from SOURCE
# under extra flags -> flashws_amd/lib/libfws_gpu_<tag>.so (not the product library).
# usage: tools/build_variant.sh TAG OBJ SOURCE.hip [hipcc flags...]   (OBJ e.g. unmask_kernels)
set -e
tag=$1; obj=$2; src=$3; shift 3
cd "$(dirname "$0")/../flashws_amd/csrc"
make -s -j8 >/dev/null
objs=$(make -s -p -n 2>/dev/null | sed -n 's/^OBJS := //p')
d=build_exp_$tag
rm -rf $d; mkdir -p $d
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I../../include -I. "$@" \
  -c $src -o $d/$obj.o -Rpass-analysis=kernel-resource-usage 2> $d/remarks.txt
list=""
for o in $objs; do b=$(basename $o); if [ "$b" = "$obj.o" ]; then list="$list $d/$b"; else list="$list $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libfws_gpu_$tag.so $list
echo "built ../lib/libfws_gpu_$tag.so"
