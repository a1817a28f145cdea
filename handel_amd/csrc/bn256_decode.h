// bn256_decode.h — signature decode shared by the decode kernels
// (bn256_kernels.hip) and the pairing kernel of the GT path (bn256_gt.hip),
// which decodes its own signature so the prologue can run off its critical path.
#pragma once
#include "bn256_curve.h"
#include "bn256_kernels.h"

namespace hg {

// SigBLS.UnmarshalBinary rules: go (x/crypto) takes the
// coordinates mod p, cf (cloudflare) rejects coordinates >= p; all-zero is
// infinity; otherwise the point must be on y^2 = x^3 + 3.
HG_DEV int32_t decode_g1_one(const uint8_t* m, int flavor, PointG1& P) {
  bool gx, gy;
  bool nz = false;  // some byte nonzero (all-zero = infinity)
  fp_from_be(P.x, m, &gx, &nz);
  fp_from_be(P.y, m + 32, &gy, &nz);
  int32_t code = HG_OK;
  P.inf = nz ? 0u : 1u;
  // every G1 point this API decodes is a signature: cloudflare's
  // SigBLS.UnmarshalBinary wraps the G1 error (bn256/cf/bn256.go:183-190)
  if (flavor == HG_FLAVOR_CF && (gx || gy)) {
    code = HG_ERR_SIG_CF_EXCEEDS;
  } else if (nz && !g1_on_curve(P.x, P.y)) {
    code = flavor == HG_FLAVOR_CF ? HG_ERR_SIG_CF_MALFORMED : HG_ERR_SIG_UNMARSHAL;
  }
  return code;
}


}  // namespace hg
