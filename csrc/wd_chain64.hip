// The register-chained fused Wide&Deep training step (csrc/wd_chain.hip) built for T = 64 examples per workgroup
// iteration: one workgroup of 4 waves x 16 examples (one wave per SIMD). The small-batch shape: at the reference
// batch (40, `airflow-dags/taxi_utils.py:300-345` trainer_fn's train_batch_size) the whole step is one iteration of
// one workgroup, and with half the waves every SIMD runs one wave's MFMA chain instead of two and every block
// barrier waits for 4 waves instead of 8. Same weight image, tile map and gradient slab as the T = 128 library;
// exported names end in _t64.
//
// MIFX_HIPCC_FLAGS: -fno-honor-nans -fno-honor-infinities
#define WDC_T 64
#include "wd_chain.hip"
