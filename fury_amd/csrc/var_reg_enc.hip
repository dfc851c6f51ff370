// var_reg_enc.hip — instances of the register-staged encode (schemas of <= kRegCols fields).
#define FURY_VAR_ENC
#include "var_dev.h"

namespace fury {

int launch_encode_var_reg(const VarArgs& b, const int64_t* offs, uint8_t* rows, int64_t cap,
                          int64_t nt, hipStream_t stream) {
  switch (b.ncols) {
#define FURY_REG(KK) case KK: hipLaunchKernelGGL(encode_var_reg<KK>, dim3(nt), dim3(kEncRows), 0, stream, b, offs, rows, cap); break;
    FURY_REG(1) FURY_REG(2) FURY_REG(3) FURY_REG(4) FURY_REG(5) FURY_REG(6) FURY_REG(7)
    FURY_REG(8) FURY_REG(9) FURY_REG(10) FURY_REG(11) FURY_REG(12) FURY_REG(13) FURY_REG(14)
    FURY_REG(15) FURY_REG(16)
#undef FURY_REG
    default: return set_error(FURY_ERR_UNSUPPORTED, "register-staged encode: 1..16 fields");
  }
  return check_hip(hipGetLastError(), "encode_var_reg launch");
}

}  // namespace fury
