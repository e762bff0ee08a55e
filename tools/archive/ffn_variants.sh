#!/bin/bash
# Build diagnostic variants of libmlgate.so that differ only in how lg_ffn.hip is compiled
# (tools/ffn_interference.py A/B): ab_ffn_slp (-fno-slp-vectorize), ab_ffn_pad (32 wait
# states after each GEMM phase), ab_ffn_both.  Run from the repo root after `make`.
set -e
C=multi-level-indoor-slam_amd/csrc
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result"
OBJS=$(ls $C/build/*.o | grep -v lg_ffn)
for v in slp pad both; do
  extra=""
  [ $v = slp ] && extra="-fno-slp-vectorize"
  [ $v = pad ] && extra="-DMLG_FFN_PAD=1"
  [ $v = both ] && extra="-fno-slp-vectorize -DMLG_FFN_PAD=1"
  mkdir -p ab_ffn_$v
  /opt/rocm/bin/hipcc $FLAGS $extra -c $C/lg_ffn.hip -o ab_ffn_$v/lg_ffn.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ab_ffn_$v/libmlgate.so $OBJS ab_ffn_$v/lg_ffn.o -lz -lpthread
  cp multi-level-indoor-slam_amd/mlgate/libmlgate_torch.so ab_ffn_$v/
  rm ab_ffn_$v/lg_ffn.o
done
