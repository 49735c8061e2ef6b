// The corrected-precision network instance (fp16 + e4m3 cross terms, 5-board
// borderless) and the fast borderless instance compiled on their own under a register
// cap: kNNForwardCap is nn.hip's
// kNNForward with amdgpu_num_vgpr(KC_F8C_VGPR) (register pairs on gfx950: 96 = 192
// VGPRs), so that a 128-VGPR search wave of the other game group fits on each SIMD
// beside the network's two waves.  The launch and the weight packing
// stay in nn.hip.
#define KC_NN_KERNEL kNNForwardCap
#define KC_NN_KERNEL_ATTR __attribute__((amdgpu_num_vgpr(KC_F8C_VGPR)))
#define KC_NN_KERNEL_ONLY
#include "nn.hip"

namespace kc {
#if KC_F8C_VGPR
template __global__ void kNNForwardCap<5, 5, 96, NN_SMALL_NB, NN_MODE_F8C, true>(
    const NNLayout* __restrict__, const h16x8* __restrict__, const float* __restrict__, const uint16_t* __restrict__,
    int, const int* __restrict__, const int* __restrict__, int, float, const uint64_t* __restrict__, float* __restrict__,
    float* __restrict__, int* __restrict__);
// the fast borderless instance under the same cap (218 VGPRs uncapped)
template __global__ void kNNForwardCap<5, 5, 96, NN_SMALL_NB, NN_MODE_F16, true>(
    const NNLayout* __restrict__, const h16x8* __restrict__, const float* __restrict__, const uint16_t* __restrict__,
    int, const int* __restrict__, const int* __restrict__, int, float, const uint64_t* __restrict__, float* __restrict__,
    float* __restrict__, int* __restrict__);
#if KC_ACC_CAP
// the accurate (split) borderless instance under the same cap (222 VGPRs uncapped)
template __global__ void kNNForwardCap<5, 5, 96, NN_SMALL_NB, NN_MODE_SPLIT3, true>(
    const NNLayout* __restrict__, const h16x8* __restrict__, const float* __restrict__, const uint16_t* __restrict__,
    int, const int* __restrict__, const int* __restrict__, int, float, const uint64_t* __restrict__, float* __restrict__,
    float* __restrict__, int* __restrict__);
#endif
#endif
}  // namespace kc
