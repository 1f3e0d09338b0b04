// mbls_status.cpp — the message text of every status code (include/mbls.h), host-only so the
// NIF shims' sanitizer builds (tests/test_sanitizers.py) link the same strings as libmbls.
// The strings are the reference NIF's `format!("{:?}", err)` renderings (SURVEY.md App. A;
// native/bls_nif/src/lib.rs:7-12 maps every Err to {:error, <that string>}).
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "../../include/mbls.h"

extern "C" {

size_t mbls_status_message(int32_t code, size_t got, char* out, size_t out_len) {
  char tmp[160];
  switch (code) {
    case MBLS_ERR_BAD_ENCODING: std::snprintf(tmp, sizeof tmp, "BlstError(BLST_BAD_ENCODING)"); break;
    case MBLS_ERR_NOT_ON_CURVE: std::snprintf(tmp, sizeof tmp, "BlstError(BLST_POINT_NOT_ON_CURVE)"); break;
    case MBLS_ERR_NOT_IN_GROUP: std::snprintf(tmp, sizeof tmp, "BlstError(BLST_POINT_NOT_IN_GROUP)"); break;
    case MBLS_ERR_PK_IS_INFINITY: std::snprintf(tmp, sizeof tmp, "BlstError(BLST_PK_IS_INFINITY)"); break;
    case MBLS_ERR_INFINITY_PUBKEY: std::snprintf(tmp, sizeof tmp, "InvalidInfinityPublicKey"); break;
    case MBLS_ERR_PUBKEY_LENGTH:
      std::snprintf(tmp, sizeof tmp, "InvalidByteLength { got: %zu, expected: 48 }", got);
      break;
    case MBLS_ERR_MESSAGE_LENGTH:
      std::snprintf(tmp, sizeof tmp, "InvalidMessageLength { got: %zu, expected: 32 }", got);
      break;
    case MBLS_ERR_EMPTY_SIGNATURES: std::snprintf(tmp, sizeof tmp, "Empty signature vector"); break;
    case MBLS_ERR_EMPTY_PUBKEYS: std::snprintf(tmp, sizeof tmp, "Empty public key vector"); break;
    case MBLS_ERR_SECRET_KEY_LENGTH:
      std::snprintf(tmp, sizeof tmp, "InvalidSecretKeyLength { got: %zu, expected: 32 }", got);
      break;
    case MBLS_ERR_ZERO_SECRET_KEY: std::snprintf(tmp, sizeof tmp, "InvalidZeroSecretKey"); break;
    case MBLS_ERR_UNKNOWN_INDEX: std::snprintf(tmp, sizeof tmp, "UnknownValidatorIndex"); break;
    case MBLS_ERR_DEVICE: std::snprintf(tmp, sizeof tmp, "DeviceError"); break;
    case MBLS_ERR_ARGUMENT: std::snprintf(tmp, sizeof tmp, "ArgumentError"); break;
    case MBLS_ERR_SCRATCH_PLAN: std::snprintf(tmp, sizeof tmp, "ScratchPlanUnavailable"); break;
    default: std::snprintf(tmp, sizeof tmp, "UnknownError(%d)", (int)code); break;
  }
  const size_t n = std::strlen(tmp);
  if (out && out_len) {
    const size_t c = std::min(n, out_len - 1);
    std::memcpy(out, tmp, c);
    out[c] = 0;
  }
  return n;
}

}  // extern "C"
