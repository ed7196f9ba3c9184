#!/bin/bash
# diagnostic (s_memtime) builds of the fused W&D kernels, same flags as the production builds
cd "$(dirname "$0")/.." && mkdir -p tools/bin && hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWD_STAMPS \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wide_deep.hip | cut -d: -f2-) -o tools/bin/libwd_stamps.so csrc/wide_deep.hip && \
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain.hip | cut -d: -f2-) -o tools/bin/libwdc_stamps.so csrc/wd_chain.hip && \
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS -Icsrc \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain64.hip | cut -d: -f2-) -o tools/bin/libwdc64_stamps.so csrc/wd_chain64.hip && \
hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS -Icsrc \
  $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain.hip | cut -d: -f2-) -o tools/bin/libwdc256_stamps.so csrc/wd_chain256.hip || exit 1
# prologue split (wrong results): the same builds without the weight-image load -- stamps_wdc.py --noimg
[ "$1" = "--noimg" ] && for v in "wd_chain.hip libwdc_noimg" "wd_chain64.hip libwdc64_noimg" "wd_chain256.hip libwdc256_noimg"; do
  set -- $v
  hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS -DWDC_DIAG_NOIMG=1 -Icsrc \
    $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain.hip | cut -d: -f2-) -o tools/bin/$2_stamps.so csrc/$1 || exit 1
done
exit 0
