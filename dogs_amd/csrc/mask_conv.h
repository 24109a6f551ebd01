// mask_conv.h -- the appearance embedding's 3x3 convolution weight gradient (mask_conv.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace gs {
// dW [Cout][Cin][3][3] and db [Cout] of a stride-1, zero-pad-1 3x3 convolution of x [Cin][H][W] with output gradient
// dy [Cout][H][W]; scratch: conv3x3_wgrad_scratch_bytes(...) bytes of per-block partials.  Deterministic.
size_t conv3x3_wgrad_scratch_bytes(int Cin, int Cout, int H, int W);
bool conv3x3_wgrad_supported(int Cin, int Cout);
void launch_conv3x3_wgrad(int Cin, int Cout, int H, int W, const float* x, const float* dy, float* dw, float* db,
                          float* scratch, hipStream_t st);
}  // namespace gs
