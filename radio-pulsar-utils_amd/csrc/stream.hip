// CU-masked compute streams for overlapping the search with RCCL.
//
// The subband search holds one 160 KiB-LDS workgroup on every CU for ~1 ms at a time;
// an RCCL broadcast launched on another stream then waits for CUs to drain before its
// own workgroups run.  A compute stream that leaves a few CUs out of its mask keeps
// those CUs free for the collective while chunks are in flight.
#include <hip/hip_runtime.h>

#include <vector>

#include "pu_common.h"

extern "C" {

int pu_stream_create_cu_masked(int reserve, void **out)
{
    PU_REQUIRE(out != nullptr, "pu_stream_create_cu_masked: out is NULL");
    *out = nullptr;
    int dev = 0;
    PU_TRY_HIP(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    PU_TRY_HIP(hipGetDeviceProperties(&prop, dev));
    const int ncu = prop.multiProcessorCount;
    PU_REQUIRE(reserve >= 0 && reserve < ncu, "pu_stream_create_cu_masked: reserve %d of %d CUs", reserve, ncu);
    std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
    for (int i = 0; i < ncu; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    // reserved CUs: one per block of ncu / reserve, stepping by one more each block, so
    // they spread over the XCDs whether the mask enumerates CUs XCD by XCD or round-robin
    // across XCDs (256 CUs, 8 reserved: CUs 0, 33, 66, ..., 231)
    if (reserve > 0) {
        const int step = ncu / reserve;
        for (int k = 0; k < reserve; ++k) {
            const int cu = k * step + (k % step);
            mask[(size_t)cu / 32] &= ~(1u << (cu % 32));
        }
    }
    hipStream_t s = nullptr;
    PU_TRY_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    *out = s;
    return PU_OK;
}

int pu_stream_destroy(void *stream)
{
    if (!stream) return PU_OK;
    PU_TRY_HIP(hipStreamDestroy(pu::as_stream(stream)));
    return PU_OK;
}

}  // extern "C"
