#!/bin/bash
# diagnostic (s_memtime) build of the fused W&D kernel, same flags as the production build
cd "$(dirname "$0")/.." && mkdir -p tools/bin && hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWD_STAMPS \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wide_deep.hip | cut -d: -f2-) -o tools/bin/libwd_stamps.so csrc/wide_deep.hip
