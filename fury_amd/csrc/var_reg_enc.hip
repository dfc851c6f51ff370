// var_reg_enc.hip — instances of the register-staged encode: K = 2, 3, 4, 6, 8, 12, 16 columns
// (reg_dec_k) x kind mode (kind_of).
#define FURY_VAR_ENC
#include "var_dev.h"

namespace fury {

int launch_measure_tiles(const VarArgs& b, int64_t* tsum, int64_t nt, hipStream_t stream) {
  hipLaunchKernelGGL(measure_tiles, dim3(static_cast<unsigned>((nt + kThreads / 64 - 1) / (kThreads / 64))),
                     dim3(kThreads), 0, stream, b, tsum, b.tile_rows, nt);
  return check_hip(hipGetLastError(), "measure_tiles launch");
}

int launch_encode_var_reg(const VarArgs& b, int64_t* offs, uint8_t* rows, int64_t cap,
                          int64_t nt, int mode, const int64_t* tbase, hipStream_t stream) {
#define FURY_REG_M(KK, M) \
  hipLaunchKernelGGL((encode_var_reg<KK, M>), dim3(nt), dim3(kEncRows), 0, stream, b, offs, rows, cap, tbase);
#define FURY_REG(KK)                                                                           \
  case KK:                                                                                     \
    if (mode == kSeqBytes) { FURY_REG_M(KK, kSeqBytes) }                                       \
    else if (mode == kSeqLists) { FURY_REG_M(KK, kSeqLists) }                                  \
    else { FURY_REG_M(KK, kSeqAll) }                                                           \
    break;
  // records b.col[0, K) come from the argument block (zero past ncols), never a device table
  if (b.tab || b.ncols > kRegCols)
    return set_error(FURY_ERR_INVALID_ARGUMENT, "register-staged encode: 1..16 fields, argument-block records");
  switch (reg_dec_k(b.ncols)) {
    FURY_REG(2) FURY_REG(3) FURY_REG(4) FURY_REG(6) FURY_REG(8) FURY_REG(12) FURY_REG(16)
    default: return set_error(FURY_ERR_UNSUPPORTED, "register-staged encode: 1..16 fields");
  }
#undef FURY_REG
#undef FURY_REG_M
  return check_hip(hipGetLastError(), "encode_var_reg launch");
}

}  // namespace fury
