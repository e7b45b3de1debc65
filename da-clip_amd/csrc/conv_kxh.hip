// conv_kxh.hip — f16 instantiations of the 1x1 / 4x4-s2 / 7x7 / patch-embed convs (split for
// parallel builds).
#include "conv_impl.h"

namespace dac {
template void conv_dispatch<f16, 1, 1, 1, 0>(const ConvArgs&, hipStream_t);
template void conv_dispatch<f16, 4, 4, 2, 1>(const ConvArgs&, hipStream_t);
template void conv_dispatch<f16, 7, 7, 1, 3>(const ConvArgs&, hipStream_t);
template void conv_dispatch<f16, 32, 32, 32, 0>(const ConvArgs&, hipStream_t);
template void conv_dispatch<f16, 14, 14, 14, 0>(const ConvArgs&, hipStream_t);
}  // namespace dac
