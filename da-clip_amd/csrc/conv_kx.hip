// conv_kx.hip — explicit instantiations of the implicit-GEMM conv (split for parallel builds).
#include "conv_impl.h"

namespace dac {
template void conv_dispatch<float, 4, 4, 2, 1>(const ConvArgs&, hipStream_t);
template void conv_dispatch<bf16, 4, 4, 2, 1>(const ConvArgs&, hipStream_t);
template void conv_dispatch<float, 7, 7, 1, 3>(const ConvArgs&, hipStream_t);
template void conv_dispatch<bf16, 7, 7, 1, 3>(const ConvArgs&, hipStream_t);
template void conv_dispatch<float, 32, 32, 32, 0>(const ConvArgs&, hipStream_t);
template void conv_dispatch<bf16, 32, 32, 32, 0>(const ConvArgs&, hipStream_t);
template void conv_dispatch<float, 14, 14, 14, 0>(const ConvArgs&, hipStream_t);
template void conv_dispatch<bf16, 14, 14, 14, 0>(const ConvArgs&, hipStream_t);
}  // namespace dac
