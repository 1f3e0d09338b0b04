// mbls_codes.h — per-element status codes shared by the kernels, the host engine and the
// host-only staging helpers (mbls_host.hpp); no HIP dependency.
#pragma once

// per-element decode codes written by the kernels (see mbls_curve.hpp DEC_*)
#define MBLS_DEC_OK 0
#define MBLS_DEC_BAD_ENCODING 1
#define MBLS_DEC_NOT_ON_CURVE 2
#define MBLS_DEC_NOT_IN_GROUP 3
#define MBLS_DEC_INFINITY 4  // exact 0xc0 00.. encoding
#define MBLS_DEC_NONE 5      // all-zero 96-byte signature (lighthouse NONE_SIGNATURE)
#define MBLS_DEC_SIG_NOT_IN_G2 6
#define MBLS_DEC_PK_LENGTH 7  // host-detected: public key binary not 48 bytes
#define MBLS_DEC_UNKNOWN_INDEX 8  // pubkey-table row never set (or index past the table)
#define MBLS_AGG_INFINITY 10  // aggregated public key is the identity
#define MBLS_AGG_EMPTY 11     // set has no keys
#define MBLS_SET_FALSE 100    // host-detected: verdict is {:ok, false} (aggregate_verify count mismatch)
