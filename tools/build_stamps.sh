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
# prologue split (wrong results): the same builds without the weight-image load (--noimg) or without the
# step-counter load ahead of the record fetch (--nostep) -- stamps_wdc.py --noimg / --nostep
case "$1" in --noimg) D=WDC_DIAG_NOIMG ;; --nostep) D=WDC_DIAG_NOSTEP ;; *) exit 0 ;; esac
S=${1#--}
for v in "wd_chain.hip libwdc" "wd_chain64.hip libwdc64" "wd_chain256.hip libwdc256"; do
  set -- $v
  hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWDC_STAMPS -D$D=1 -Icsrc \
    $(grep '^// MIFX_HIPCC_FLAGS:' csrc/wd_chain.hip | cut -d: -f2-) -o tools/bin/$2_${S}_stamps.so csrc/$1 || exit 1
done
exit 0
