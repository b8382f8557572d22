#!/bin/bash
# gfx950 assembly of one translation unit (count_pipnet_amd/csrc/<tu>.hip, or tools/<tu>.hip) with the
# product flags, into /tmp/isa_<tu>.s -- for reading a kernel's s_waitcnt / store forms.
#   tools/isa_dump.sh gemm_f32
set -eu
tu=$1
R=$(cd "$(dirname "$0")/.." && pwd)
src="$R/count_pipnet_amd/csrc/$tu.hip"
[ -f "$src" ] || src="$R/tools/$tu.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --offload-device-only -S -o "/tmp/isa_$tu.s" "$src" \
  -I "$R/include" 2>&1 | grep -v "warning" || true
echo "/tmp/isa_$tu.s"
