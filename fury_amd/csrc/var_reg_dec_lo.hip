// var_reg_dec_lo.hip — instances of the register-staged decode for 1..8 fields.
#define FURY_VAR_DEC
#include "var_dev.h"

namespace fury {

int launch_decode_var_reg(const VarArgs& a, const uint8_t* rows, const int64_t* offs, uint64_t* status,
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
    FURY_DREG(1) FURY_DREG(2) FURY_DREG(3) FURY_DREG(4) FURY_DREG(5) FURY_DREG(6) FURY_DREG(7) FURY_DREG(8)
#undef FURY_DREG
    default: return launch_decode_var_reg_hi(a, rows, offs, status, img, wide, nb, nbr, stream);
  }
  return check_hip(hipGetLastError(), "decode_var_reg launch");
}

}  // namespace fury
