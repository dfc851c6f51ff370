// var_reg_dec_hi.hip — instances of the register-staged decode for K = 8, 12, 16 (reg_dec_k), every
// kind mode (kind_of).
#define FURY_VAR_DEC
#include "var_dev.h"

namespace fury {

#define FURY_DREG_M(KK, M)                                                                     \
  if (a.dec_pipe && dec_pipe_k(KK)) {                                                          \
    const size_t lds = img + 2 * static_cast<size_t>(stage);                                   \
    const void* kf = reinterpret_cast<const void*>(decode_var_reg<KK, M, dec_pipe_k(KK)>);     \
    hipLaunchKernelGGL((decode_var_reg<KK, M, dec_pipe_k(KK)>), dim3(dec_pipe_grid(kf, nt, lds)), \
                       dim3(kDecThreads), lds, stream, a, rows, offs, status, img, stage);     \
  } else {                                                                                     \
    hipLaunchKernelGGL((decode_var_reg<KK, M>), dim3(nt), dim3(kDecThreads), img + stage, stream, \
                       a, rows, offs, status, img, stage);                                     \
  }
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

}  // namespace fury
