// conv_k3h.hip — f16 instantiation of the 3x3 implicit-GEMM conv (split for parallel builds).
#include "conv_impl.h"

namespace dac {
template void conv_dispatch<f16, 3, 3, 1, 1>(const ConvArgs&, hipStream_t);
}  // namespace dac
