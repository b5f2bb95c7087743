#!/bin/bash
# A/B library: csrc/libmmfusion_<tag>.so = the product objects with ONE source file taken from
# another git revision (or the work tree: rev "-") and/or built with extra flags, for alternating
# bench runs under MMF_LIB_PATH on one box.
# The other objects are the ones already built (run `make` first): the product library itself is
# not rebuilt, so a GPU call in flight keeps the tree it was sent with.
# usage: scripts/build_ab_lib.sh <file.hip> <tag> [rev|-] [extra hipcc flags...]
set -euo pipefail
cd "$(dirname "$0")/../multimodal-sensor-fusion-with-attention-rajeevatla_amd/csrc"
F=${1:?source file}; TAG=${2:?tag}; REV=${3:-HEAD}
shift 3 || shift $#
B=${F%.hip}
if [ "$REV" = "-" ]; then cp "$F" "/tmp/${B}_${TAG}.hip"; else git show "$REV:./$F" > "/tmp/${B}_${TAG}.hip"; fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../../include -I. "$@" \
  -c "/tmp/${B}_${TAG}.hip" -o "/tmp/${B}_${TAG}.o"
objs=$(echo $(make -s -p -n all 2>/dev/null | sed -n 's/^OBJS := //p' | head -1))
[ -n "$objs" ] || objs="gemm.o attention.o head.o pool.o tail.o hybrid.o capi.o softmax_pool.o chunks.o lstm.o single_key.o wide.o attn_long.o l1.o"
objs=$(for o in $objs; do [ "$o" = "$B.o" ] || echo $o; done)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "libmmfusion_${TAG}.so" $objs "/tmp/${B}_${TAG}.o"
echo "libmmfusion_${TAG}.so: $F from $REV $*"
