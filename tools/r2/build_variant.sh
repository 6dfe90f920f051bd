#!/bin/bash
# Build a variant of libhwy.so with extra compile flags (development A/B):
#   build_variant.sh <tag> <flags...>  ->  highway-rope-ppo_amd/hwy/libhwy_<tag>.so
set -e
TAG=$1; shift
C=$(dirname $0)/../../highway-rope-ppo_amd/csrc
B=$(dirname $0)/../../build/csrc
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -Wall -I$C/../../include -I$C -fno-gpu-rdc"
/opt/rocm/bin/hipcc $F "$@" -c $C/ppo_kernels.hip -o $B/ppo_kernels_$TAG.o
/opt/rocm/bin/hipcc $F "$@" -c $C/hwy_kernels.hip -o $B/hwy_kernels_$TAG.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $C/../hwy/libhwy_$TAG.so $B/hwy_kernels_$TAG.o $B/ppo_kernels_$TAG.o $B/hwy_api.o
