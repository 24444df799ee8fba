#!/bin/bash
# Timing ablations of the relative-key dK/dV kernel (STE_ABLATE bit mask, see attention.hip):
# builds speech_transcript_embeddings_amd/_abl/libste_abl<mask>.so here (CPU), then on the GPU:
#   for m in ...; do STE_LIB=.../libste_abl$m.so python3 profiles/attn_probe.py; done
set -e
cd "$(dirname "$0")/.."
PKG=speech_transcript_embeddings_amd
mkdir -p $PKG/_abl
for m in "$@"; do
  objs=()
  for f in $PKG/_obj/*.o; do
    [ "$(basename $f)" = attention.o ] || objs+=("$f")
  done
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Iinclude -I$PKG/csrc \
    -DSTE_ABLATE=$m -c $PKG/csrc/attention.hip -o $PKG/_abl/attention_$m.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/_abl/libste_abl$m.so "${objs[@]}" $PKG/_abl/attention_$m.o
done
