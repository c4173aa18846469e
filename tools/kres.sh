#!/bin/bash
# Register / LDS / spill report of every kernel instantiated in one .hip file
# (device-only compile, gfx950): tools/kres.sh csrc/kernels/stencil_tbl.hip [extra clang flags]
f=${1:-csrc/kernels/stencil_tbl.hip}; shift
/opt/rocm/llvm/bin/clang++ -DUSE_PROF_API=1 -D__HIP_PLATFORM_AMD__=1 -I"$(dirname "$0")/../csrc" -O3 -std=gnu++17 \
  --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -x hip -c "$f" --offload-device-only -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | sed -n 's/.*remark: *\(.*\) \[-Rpass-analysis.*/\1/p' |
  awk '/^Function Name:/{n=$NF} /^VGPRs:/{v=$NF} /^ScratchSize/{s=$NF} /^SGPRs Spill:/{ss=$NF} /^VGPRs Spill:/{vs=$NF}
       /^LDS Size/{l=$NF; print n, "vgpr="v, "scratch="s, "sgpr_spill="ss, "vgpr_spill="vs, "lds="l}' |
  c++filt | sed 's/void heat3d::hip:://; s/([^)]*)//'
