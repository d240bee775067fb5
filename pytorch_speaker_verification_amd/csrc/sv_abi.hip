// dtype-enum entry points of the stack (include/sv_ge2e.h, "dtype-enum form"): one entry point per
// direction with the precision as an argument, as SURVEY.md §8 b specifies the boundary
// (`lstm_fwd` = K1 + K2, `lstm_bwd` = K3 + K4).  Host code only: each call forwards to the
// dtype-specific stack function, which does the work (sv_lstm.hip / sv_bf16.hip / sv_persist*.hip).
#include "sv_common.h"
#include "../../include/sv_ge2e.h"

extern "C" int sv_lstm_fwd(int dtype, int L, int T, int B, int F, int H, const void* x, const void* const* w_ih,
                           const void* const* w_hh, const float* const* b_ih, const float* const* b_hh,
                           void* const* gates, float* const* c_tm, float* const* h_tm, void* const* h_bf,
                           void* const* hT, int chunk, hipStream_t main, const hipStream_t* side, hipEvent_t* ev,
                           int products, int schedule, void* sync, hipEvent_t* probe) {
  switch (dtype) {
    case SV_DTYPE_F32:
      return sv_lstm_stack_fwd(L, T, B, F, H, static_cast<const float*>(x),
                               reinterpret_cast<const float* const*>(w_ih), reinterpret_cast<const float* const*>(w_hh),
                               b_ih, b_hh, reinterpret_cast<float* const*>(gates), c_tm, h_tm,
                               reinterpret_cast<float* const*>(hT), chunk, main, side, ev, products, schedule,
                               static_cast<unsigned*>(sync), probe);
    case SV_DTYPE_BF16:
      return sv_lstm_stack_fwd_bf16(L, T, B, F, H, static_cast<const sv_bf16*>(x),
                                    reinterpret_cast<const sv_bf16* const*>(w_ih),
                                    reinterpret_cast<const sv_bf16* const*>(w_hh), b_ih, b_hh,
                                    reinterpret_cast<sv_bf16* const*>(gates), c_tm, h_tm,
                                    reinterpret_cast<sv_bf16* const*>(h_bf), reinterpret_cast<sv_bf16* const*>(hT),
                                    chunk, main, side, ev, sync, probe, schedule);
    default:
      return SV_EARG;
  }
}

extern "C" size_t sv_lstm_bwd_workspace(int dtype, int L, int T, int B, int F, int H) {
  switch (dtype) {
    case SV_DTYPE_F32:
      return sv_lstm_stack_bwd_workspace(L, T, B, F, H);
    case SV_DTYPE_BF16:
      return sv_lstm_stack_bwd_bf16_workspace(L, T, B, F, H);
    default:
      return 0;
  }
}

extern "C" int sv_lstm_bwd(int dtype, int L, int T, int B, int F, int H, const void* const* xT, const long* ld_xT,
                           const float* const* w_ih, const float* const* w_hh, const void* const* gates,
                           const float* const* c_tm, const void* const* hT, const float* dh_last, void* const* dg,
                           void* const* dgT, float* const* dx, float* const* dw_ih, float* const* dw_hh,
                           float* const* db_ih, float* const* db_hh, void* workspace, int chunk, hipStream_t main,
                           const hipStream_t* side, hipEvent_t* ev, int products, hipEvent_t* probe,
                           unsigned long long* kstamp, int schedule, void* sync) {
  switch (dtype) {
    case SV_DTYPE_F32:
      return sv_lstm_stack_bwd(L, T, B, F, H, reinterpret_cast<const float* const*>(xT), ld_xT, w_ih, w_hh,
                               reinterpret_cast<const float* const*>(gates), c_tm,
                               reinterpret_cast<const float* const*>(hT), dh_last, reinterpret_cast<float* const*>(dg),
                               reinterpret_cast<float* const*>(dgT), dx, dw_ih, dw_hh, db_ih, db_hh,
                               static_cast<float*>(workspace), chunk, main, side, ev, products, probe, kstamp, schedule,
                               static_cast<unsigned*>(sync));
    case SV_DTYPE_BF16:
      return sv_lstm_stack_bwd_bf16(L, T, B, F, H, reinterpret_cast<const sv_bf16* const*>(xT), ld_xT, w_ih, w_hh,
                                    reinterpret_cast<const sv_bf16* const*>(gates), c_tm,
                                    reinterpret_cast<const sv_bf16* const*>(hT), dh_last,
                                    reinterpret_cast<sv_bf16* const*>(dg), reinterpret_cast<sv_bf16* const*>(dgT), dx,
                                    dw_ih, dw_hh, db_ih, db_hh, workspace, chunk, main, side, ev, sync, probe, schedule);
    default:
      return SV_EARG;
  }
}
