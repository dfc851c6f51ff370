// var_reg_dec_hi.hip — instances of the register-staged decode for K = 8, 12, 16 (reg_dec_k) and the
// column-chunked one for wider schemas, every kind mode (kind_of).
#define FURY_VAR_DEC
#include "var_dev.h"

namespace fury {

#define FURY_DREG_M(KK, M)                                                                     \
  hipLaunchKernelGGL((decode_var_reg<KK, M>), dim3(nt), dim3(kDecThreads), img + stage, stream, a, \
                     rows, offs, status, img, stage);
#define FURY_DREG(KK)                                                                          \
  case KK:                                                                                     \
    if (mode == kSeqBytes) { FURY_DREG_M(KK, kSeqBytes) }                                      \
    else if (mode == kSeqLists) { FURY_DREG_M(KK, kSeqLists) }                                 \
    else { FURY_DREG_M(KK, kSeqAll) }                                                          \
    break;

int launch_decode_var_reg_hi(const VarArgs& a, const uint8_t* rows, const int64_t* offs, uint64_t* status,
                             uint32_t img, uint32_t stage, int mode, int64_t nt, hipStream_t stream) {
  switch (reg_dec_k(a.ncols)) {
    FURY_DREG(8) FURY_DREG(12) FURY_DREG(16)
    default: return set_error(FURY_ERR_UNSUPPORTED, "register-staged decode: 1..16 fields");
  }
  return check_hip(hipGetLastError(), "decode_var_reg launch");
}

int launch_decode_var_reg_wide(const VarArgs& a, const uint8_t* rows, const int64_t* offs,
                               uint64_t* status, uint32_t img, uint32_t stage, int mode, int64_t nt,
                               int kc, hipStream_t stream) {
#define FURY_DREG_W(KC, M)                                                                     \
  hipLaunchKernelGGL((decode_var_reg<KC, M, true>), dim3(nt), dim3(kDecThreads), img + stage,    \
                     stream, a, rows, offs, status, img, stage);
#define FURY_DREG_WK(KC)                                                                       \
  if (kc == KC) {                                                                              \
    if (mode == kSeqBytes) { FURY_DREG_W(KC, kSeqBytes) }                                      \
    else if (mode == kSeqLists) { FURY_DREG_W(KC, kSeqLists) }                                 \
    else { FURY_DREG_W(KC, kSeqAll) }                                                          \
    return check_hip(hipGetLastError(), "decode_var_reg (chunked) launch");                    \
  }
  FURY_DREG_WK(4)
  FURY_DREG_WK(8)
  FURY_DREG_WK(16)
#undef FURY_DREG_WK
#undef FURY_DREG_W
  return set_error(FURY_ERR_INVALID_ARGUMENT, "chunked decode: 4, 8 or 16 fields per chunk");
}

}  // namespace fury
