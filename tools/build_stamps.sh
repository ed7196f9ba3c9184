#!/bin/bash
# diagnostic (s_memtime) builds of the fused W&D kernels, same flags as the production builds
cd "$(dirname "$0")/.." && mkdir -p tools/bin && hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWD_STAMPS \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wide_deep.hip | cut -d: -f2-) -o tools/bin/libwd_stamps.so csrc/wide_deep.hip && \
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain.hip | cut -d: -f2-) -o tools/bin/libwdc_stamps.so csrc/wd_chain.hip && \
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS -Icsrc \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain64.hip | cut -d: -f2-) -o tools/bin/libwdc64_stamps.so csrc/wd_chain64.hip && \
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS -Icsrc \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain.hip | cut -d: -f2-) -o tools/bin/libwdc256_stamps.so csrc/wd_chain256.hip
