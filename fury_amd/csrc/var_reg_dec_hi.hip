// var_reg_dec_hi.hip — instances of the register-staged decode for 9..16 fields.
#define FURY_VAR_DEC
#include "var_dev.h"

namespace fury {

int launch_decode_var_reg_hi(const VarArgs& a, const uint8_t* rows, const int64_t* offs, uint64_t* status,
                             uint32_t img, bool wide, int64_t nb, int64_t nbr,
                             hipStream_t stream) {
  switch (a.ncols) {
#define FURY_DREG(KK)                                                                          \
  case KK:                                                                                     \
    if (wide)                                                                                  \
      hipLaunchKernelGGL((decode_var_reg<KK, 512>), dim3(nbr), dim3(512), img, stream, a,      \
                         rows, offs, status, img);                                     \
    else                                                                                       \
      hipLaunchKernelGGL(decode_var_reg<KK>, dim3(nb), dim3(kThreads), img, stream, a, rows,   \
                         offs, status, img);                                           \
    break;
    FURY_DREG(9) FURY_DREG(10) FURY_DREG(11) FURY_DREG(12) FURY_DREG(13) FURY_DREG(14) FURY_DREG(15) FURY_DREG(16)
#undef FURY_DREG
    default: return set_error(FURY_ERR_UNSUPPORTED, "register-staged decode: 1..16 fields");
  }
  return check_hip(hipGetLastError(), "decode_var_reg launch");
}

}  // namespace fury
