// sweep_wavefront.hpp -- pipelined column-wavefront sweep (placeholder: not yet enabled).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace sdfhip {
struct WavefrontWorkspace {
    int dummy = 0;
};
inline bool wavefront_supported(int, int, int) { return false; }
inline int wavefront_sweep(WavefrontWorkspace &, hipStream_t, const float4 *, unsigned long long *, const float *,
                           float, int, int, int, int, int, int, char *, size_t)
{
    return -4;
}
inline void wavefront_release(WavefrontWorkspace &) {}
}  // namespace sdfhip
