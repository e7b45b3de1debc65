// conv_k3.hip — explicit instantiations of the implicit-GEMM conv (split for parallel builds).
#include "conv_impl.h"

namespace dac {
template void conv_dispatch<float, 3, 3, 1, 1>(const ConvArgs&, hipStream_t);
template void conv_dispatch<bf16, 3, 3, 1, 1>(const ConvArgs&, hipStream_t);
}  // namespace dac
