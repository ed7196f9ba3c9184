// The register-chained fused Wide&Deep training step (csrc/wd_chain.hip) built for T = 256 examples per workgroup
// iteration: 8 waves x 32 examples (two 16-example column blocks per wave, like the 4-wave T = 128 shape, at two waves
// per SIMD). The large-batch shape: at B = 65536 on 256 workgroups each workgroup runs ONE iteration instead of two,
// so the dependent forward / activation-gradient chains of its 256 examples run once, with both column blocks'
// MFMAs interleaved in each wave, and the per-iteration fixed costs (record fetch, wide gather, loss, barriers of
// the unsplit layers) are paid once. Layers 1-3 stage their dW operands in two passes of 128 rows (the full
// 256-row staging does not fit next to the weight image in 160 KB of LDS). Same weight image, tile map and
// gradient slab as the T = 128 library; exported names end in _t256.
//
// MIFX_HIPCC_FLAGS: -fno-honor-nans -fno-honor-infinities
#define WDC_T 256
#include "wd_chain.hip"
