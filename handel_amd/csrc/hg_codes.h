// hg_codes.h — the reference's error text for every hg_code (shared by
// libhandel_gpu.so and libhandel_client.so, which must not depend on it).
#pragma once
#include "../../include/handel_gpu.h"

namespace hg {

inline const char* code_text(int code, int flavor) {
  switch (code) {
    case HG_OK: return "";
    case HG_ERR_SIG_INVALID: return "bn256: signature invalid";
    case HG_ERR_HASH_EOF: return "EOF";
    case HG_ERR_LEVEL: return "handel: inconsistent bitset with given level";
    case HG_ERR_PK_UNMARSHAL: return "unable to unmarshal";
    case HG_ERR_SIG_UNMARSHAL: return flavor == HG_FLAVOR_CF ? "bn256: multisig can't unmarshal: bn256: malformed point"
                                                             : "bn256: multisig can't unmarshal";
    case HG_ERR_EMPTY_AGG: return "runtime error: invalid memory address or nil pointer dereference";
    case HG_ERR_CF_EXCEEDS: return "bn256: coordinate exceeds modulus";
    case HG_ERR_CF_MALFORMED: return "bn256: malformed point";
    case HG_ERR_CF_SHORT: return "bn256: not enough data";
    case HG_ERR_SIG_CF_EXCEEDS: return "bn256: multisig can't unmarshal: bn256: coordinate exceeds modulus";
    case HG_ERR_SIG_CF_MALFORMED: return "bn256: multisig can't unmarshal: bn256: malformed point";
    case HG_ERR_SIG_CF_SHORT: return "bn256: multisig can't unmarshal: bn256: not enough data";
    case HG_ERR_MULTI_SIZES: return "verify multisignature: inconsistent sizes";
    case HG_ERR_PKT_ORIGIN: return "packet's origin out of range";
    case HG_ERR_PKT_LEVEL: return "invalid packet's level";
    case HG_ERR_PKT_EOF: return "EOF";
    case HG_ERR_PKT_UNEXPECTED_EOF: return "unexpected EOF";
    case HG_ERR_PKT_BITSET_SHORT: return "bitset received smaller than expected";
    case HG_ERR_PKT_TYPE_MISMATCH: return "unmarshalling error: type mismatch";
    case HG_ERR_PKT_BITSET_SIZE: return "invalid bitset's size for given level";
    case HG_ERR_PKT_NO_SIG: return "no signature in the bitset";
    case HG_ERR_PKT_ID_RANGE: return "globalID outside level's range";
    case HG_PKT_NO_IND: return "";
    case HG_ERR_ARG: return "invalid argument";
    default: return "device error";
  }
}

// processing.go:361-365 wraps only VerifySignature's error: fmt.Errorf("handel: %s", err)
inline const char* processing_text(int code, int flavor) {
  switch (code) {
    case HG_ERR_SIG_INVALID: return "handel: bn256: signature invalid";
    case HG_ERR_HASH_EOF: return "handel: EOF";
    default: return code_text(code, flavor);
  }
}

}  // namespace hg
