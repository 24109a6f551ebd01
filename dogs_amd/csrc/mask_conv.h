// mask_conv.h -- the appearance embedding's 3x3 convolution weight gradient (mask_conv.hip)
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace gs {
// dW [Cout][Cin][3][3] and db [Cout] of a stride-1, zero-pad-1 3x3 convolution of x [Cin][H][W] with output gradient
// dy [Cout][H][W]; scratch: conv3x3_wgrad_scratch_bytes(...) bytes of per-block partials.  Deterministic.
size_t conv3x3_wgrad_scratch_bytes(int Cin, int Cout, int H, int W);
bool conv3x3_wgrad_supported(int Cin, int Cout);
// column sums of per-block partials [nrows][ncols] in a fixed order; seg: rowsum_scratch_floats(nrows, ncols) floats;
// columns < nsplit go to out_a, the rest to out_b
size_t rowsum_scratch_floats(int nrows, int ncols);
void launch_rowsum(const float* part, int nrows, int ncols, float* seg, float* out_a, int nsplit, float* out_b,
                   hipStream_t st);
// gate (may be nullptr): dy counts only where gate > 0 (the backward of a ReLU whose output gate is, folded in)
// shuffle: x is [4 Cin][H / 2][W / 2], read as its pixel shuffle (PixelShuffle(2))
void launch_conv3x3_wgrad(int Cin, int Cout, int H, int W, const float* x, const float* dy, const float* gate,
                          bool shuffle, float* dw, float* db, float* scratch, hipStream_t st);
// y [Cout][H][W] = conv3x3(x [Cin][H][W], w [Cout][Cin][3][3]) + b (b may be null), relu: max(y, 0); adjoint: y [Cin]
// = the data gradient for dy = x [Cout] (w read transposed and flipped, b unused), gate (may be null): dy counts only
// where gate > 0.  Fixed summation order.
bool conv3x3_supported(int Cin, int Cout, int H, int W);
// shuffle: the forward's x is [4 Cin][H / 2][W / 2] read as its pixel shuffle; the adjoint's y is written unshuffled
void launch_conv3x3(int Cin, int Cout, int H, int W, const float* x, const float* w, const float* b, float* y,
                    bool adjoint, bool relu, const float* gate, bool shuffle, hipStream_t st);

// The embedding's full-resolution head (mask_head.hip): mask [3][H][W] = conv2(relu(conv1(resize(u)))), u [16][h2][w2],
// w1 [8][16][3][3], b1 [8], w2 [3][8][3][3], b2 [3]; the backward takes dmask and writes du [16][h2][w2] and the
// parameter gradients in one [mask_head_nparams()] row: dW1 | db1 | dW2 | db2.
struct HeadArgs {
    int H, W, h2, w2;
    float sh, sw;          // (float) h2 / H, (float) w2 / W (torch's scale for a size-given resize)
    const float *U, *k1, *b1, *k2, *b2;   // conv1 / conv2 weights and biases
    float* mask;           // forward output
    const float* dmask;    // backward input
    float *dh, *dx, *du, *part;   // backward scratch (dh [8][H][W], dx [16][H][W], part [tiles][nparams]) and du
    float* hid;            // the hidden layer relu(conv1(...)) [8][H][W]: written by the forward, read by the backward
                           // (nullptr: the forward stores nothing, the backward recomputes it)
    int tiles_x, tiles_y;
};
int mask_head_tiles(int H, int W);
int mask_head_nparams();
void launch_mask_head_fwd(HeadArgs a, hipStream_t st);
void launch_mask_head_bwd(HeadArgs a, float* grads, hipStream_t st);
}  // namespace gs
