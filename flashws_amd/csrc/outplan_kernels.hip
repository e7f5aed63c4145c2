// outplan_kernels.hip -- the output-space plan as a launch of its own: the
// out-of-place reassembly (fws_gpu_unmask_gather, C4: region f's payload goes
// to dst + dbase[f]) and the TX frame builder (fws_gpu_encode_frames: frame f
// goes to out + obase[f]); the block body is outplan_common.h's. Replaced a
// count / scan / unit-search sequence of three launches.
#include "fws_device.h"
#include "fws_internal.h"
#include "outplan_common.h"

namespace fwsk {

template <typename Desc, int kF>
__global__ __launch_bounds__(kBlock) void k_out_plan(const Desc *__restrict__ d, uint32_t n, OutPlanArgs a) {
    out_plan_block<Desc, kF>(d, n, a, plan_block_order(a.ticket));
}

}  // namespace fwsk

using namespace fwsk;

int fws_plan_next_epoch(fws_plan_ws &ws, hipStream_t s) {
    if (++ws.epoch > 0xFFFFu) {                       // tags wrapped: clear the words of old calls
        int r = fws_hip_status(hipMemsetAsync(ws.status, 0, ws.status_cap * 8, s));
        if (r) return r;
        ws.epoch = 1;
    }
    return 0;
}

template <typename Desc>
static int launch_out_plan(const Desc *d, uint32_t n, fws_plan_ws &ws, uint64_t out_cap, uint64_t *out_len,
                           hipStream_t s) {
    if (n == 0) return 0;
    const bool small = n <= 16384u;                   // few frames: 64 per workgroup
    const uint32_t nb = small ? (n + 63u) / 64u : (n + kBlock - 1) / kBlock;
    if (nb > ws.status_cap) return FWS_ERR_CAPACITY;
    int r = fws_plan_next_epoch(ws, s);
    if (r) return r;
    OutPlanArgs a{ws.cbase, ws.unit_first, ws.unit_cap, ws.total, out_len, out_cap, ws.status, ws.ticket, ws.epoch};
    if (small)
        hipLaunchKernelGGL((k_out_plan<Desc, 64>), dim3(nb), dim3(kBlock), 0, s, d, n, a);
    else
        hipLaunchKernelGGL((k_out_plan<Desc, kBlock>), dim3(nb), dim3(kBlock), 0, s, d, n, a);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_gather_plan(const fws_frame_desc *d, uint32_t n, fws_plan_ws &ws, hipStream_t s) {
    return launch_out_plan(d, n, ws, ~0ull, nullptr, s);
}

int fws_launch_tx_plan(const fws_tx_desc *d, uint32_t n, fws_plan_ws &ws, uint64_t out_cap, uint64_t *out_len,
                       hipStream_t s) {
    return launch_out_plan(d, n, ws, out_cap, out_len, s);
}
