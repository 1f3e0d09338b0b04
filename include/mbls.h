/*
 * mbls.h — C ABI of the MI355X BLS12-381 engine (libmbls.so).
 *
 * This is the boundary that replaces the reference's Rust NIF `native/bls_nif`
 * (native/bls_nif/src/lib.rs:14-158, loaded by `use Rustler` at lib/bls.ex:5).  Plain
 * pointers and sizes only; no torch types.  Two layers:
 *
 *  1. `mbls_bls_*` — one call per `Bls.*` function with the reference's exact semantics
 *     (argument meaning, error precedence, `{:ok, _}` / `{:error, msg}` outcome and the
 *     `format!("{:?}", bls::Error)` message), taking the Erlang binaries as (pointer, length)
 *     pairs.  These are what the C NIF shim (lambda_ethereum_consensus_amd/nif/bls_nif.c)
 *     binds; INTEGRATION.md shows the binding.  Each also has a `_batch` form that
 *     verifies many independent signature sets in one device submission (the batching
 *     queue of SURVEY.md §8f-1 calls these).
 *
 *  2. `mbls_dev_*` — fixed-size, device-resident batch entry points used by the batch
 *     layer and by bench.py (inputs already in HBM, asynchronous on a caller stream).
 *
 * Result codes (int32 per set): 1 = {:ok, true}, 0 = {:ok, false}, < 0 = {:error, msg}
 * with msg = mbls_status_message(code, ...).  Functions returning bytes (sign, aggregate,
 * eth_aggregate_pubkeys) return MBLS_OK (2) on success.
 */
#ifndef MBLS_H_
#define MBLS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mbls_status {
  MBLS_OK = 2,   /* byte-returning call succeeded                             */
  MBLS_TRUE = 1, /* {:ok, true}                                               */
  MBLS_FALSE = 0,/* {:ok, false}                                              */
  MBLS_ERR_BAD_ENCODING = -1,      /* BlstError(BLST_BAD_ENCODING)              */
  MBLS_ERR_NOT_ON_CURVE = -2,      /* BlstError(BLST_POINT_NOT_ON_CURVE)        */
  MBLS_ERR_NOT_IN_GROUP = -3,      /* BlstError(BLST_POINT_NOT_IN_GROUP)        */
  MBLS_ERR_PK_IS_INFINITY = -4,    /* BlstError(BLST_PK_IS_INFINITY)            */
  MBLS_ERR_INFINITY_PUBKEY = -5,   /* InvalidInfinityPublicKey                  */
  MBLS_ERR_PUBKEY_LENGTH = -6,     /* InvalidByteLength { got, expected: 48 }   */
  MBLS_ERR_MESSAGE_LENGTH = -7,    /* message not 32 bytes (reference panics)   */
  MBLS_ERR_EMPTY_SIGNATURES = -8,  /* "Empty signature vector"                  */
  MBLS_ERR_EMPTY_PUBKEYS = -9,     /* "Empty public key vector"                 */
  MBLS_ERR_SECRET_KEY_LENGTH = -10,/* InvalidSecretKeyLength { got, expected }  */
  MBLS_ERR_ZERO_SECRET_KEY = -11,  /* InvalidZeroSecretKey                      */
  MBLS_ERR_UNKNOWN_INDEX = -12,    /* UnknownValidatorIndex (pubkey table; no   */
                                   /* reference equivalent: additive API)       */
  MBLS_ERR_DEVICE = -100,          /* HIP failure (never a crash of the VM)     */
  MBLS_ERR_ARGUMENT = -101,        /* malformed call (NULL pointer, offsets)    */
  MBLS_ERR_SCRATCH_PLAN = -102     /* mbls_init: the device's scratch plan is not
                                      safe or cannot be set      */
};

/* An Erlang binary as the NIF sees it (enif_inspect_binary). */
typedef struct {
  const uint8_t* data;
  size_t len;
} mbls_bin;

/* ---------------------------------------------------------------- lifecycle ------- */
/* Selects the HIP device and allocates engine state; idempotent.  Called from the NIF's
 * `load` callback (the reference has no equivalent: Rustler's init!, lib.rs:147).
 * Hardware queues: the engine sizes its stream pool from GPU_MAX_HW_QUEUES as the process was
 * started with (HIP's default 4; the measured best is 10); the library never modifies the
 * process environment, so a BEAM node sets GPU_MAX_HW_QUEUES=10 in its release environment
 * (vm.args / env.sh), before the NIF is loaded.
 * Scratch: the first engine on a device lowers the runtime's scratch retain threshold of that
 * device (hsa_amd_agent_set_async_scratch_limit) to the value mbls_scratch_plan computes for
 * the process's hardware queues, and every dispatch of a kernel whose frame lies above it passes
 * the device's use-once gate, which keeps the use-once blocks live at any moment within
 * use_once_budget: retained blocks <= queues x threshold, use-once blocks <= pool - that, so
 * no mix of kernels on any queues and callers can exhaust the device's scratch pool (an exhausted
 * pool aborts the queue: HSA_STATUS_ERROR_OUT_OF_RESOURCES).  When the plan is not safe, the
 * threshold cannot be set or the limits cannot be read, mbls_init fails with
 * MBLS_ERR_SCRATCH_PLAN (and every later call with it) instead of running unguarded. */
int32_t mbls_init(int32_t device);
/* One engine per listed GPU ordinal, in one process (a BEAM node driving all GPUs of a host).
 * Must come before any other call (or after mbls_shutdown); idempotent for the same list,
 * MBLS_ERR_ARGUMENT for a different one.  Layer-1 batches (mbls_bls_*_batch, the indexed
 * batch and the queue) are then split into contiguous chunks of sets balanced by key count
 * (mbls_plan_shards) and verified on all engines at once, one host thread per engine; calls
 * too small to split go whole to one engine, round robin.  A repeated ordinal makes two
 * engines on one GPU (used by the tests to exercise the split on a one-GPU host). */
int32_t mbls_init_devices(const int32_t* devices, uint32_t n);
/* number of engines of the process (1 after mbls_init) */
int32_t mbls_engine_count(void);
/* Layer-2 calls (mbls_dev_*) of the calling thread go to engine `engine` (default 0); device
 * pointers passed to them must belong to that engine's GPU. */
int32_t mbls_dev_select(int32_t engine);
/* The split the layer-1 batches use: bounds[0] = 0 <= bounds[1] <= ... <= bounds[parts] =
 * n_sets, chunk j = sets [bounds[j], bounds[j+1]), cost-balanced with a set costing its key
 * count (key_off[s+1] - key_off[s]) plus 16 (its G2 chain); key_off == NULL: one key per set.
 * Host-only (no GPU needed); SURVEY.md §8e "contiguous chunks balanced by key count". */
int32_t mbls_plan_shards(const uint32_t* key_off, size_t n_sets, uint32_t parts, uint32_t* bounds);
/* Scratch plan (host-only, no GPU needed).  The runtime backs every hardware queue's scratch out
 * of one per-device pool of `pool_bytes` and keeps a queue's scratch, sized for a full-device
 * dispatch (frame bytes x 64 lanes x 32 wave slots x `cus`), when that is at most its retain
 * threshold; bigger needs are use-once, sized to the dispatch.  Given the kernels' frames (bytes
 * per lane), the plan picks the largest threshold -- one of the frames' needs, never above
 * `retain_default` -- with  queues x threshold + (largest frame above it, full device) <= pool.
 * `safe` is 0 when not even threshold 0 fits (one kernel's full-device frame exceeds the pool).
 * use_once_budget = pool - queues x threshold is what the engine's use-once gate lets all live
 * use-once dispatches of the device hold together (>= worst_use_once when safe). */
typedef struct mbls_scratch_plan_t {
  uint64_t pool_bytes;         /* HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX                          */
  uint64_t retain_default;     /* the runtime's threshold (HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_CURRENT) */
  uint64_t retain_bytes;       /* the planned threshold                                         */
  uint64_t worst_retained;     /* queues x largest retained per-queue need                      */
  uint64_t worst_use_once;     /* one full-device use-once dispatch of the largest larger frame */
  uint32_t queues;             /* hardware queues priced                                        */
  uint32_t max_frame;          /* largest frame of the kernels (bytes per lane)                 */
  uint32_t max_retained_frame; /* largest frame a queue keeps                                   */
  int32_t safe;                /* worst_retained + worst_use_once <= pool_bytes                 */
  int32_t applied;             /* mbls_scratch_info: the engine set retain_bytes on the device  */
  uint64_t use_once_budget;    /* pool_bytes - worst_retained: the use-once gate's bound         */
} mbls_scratch_plan_t;
/* gated (optional, one flag per frame): 1 = the engine's use-once gate admits that kernel's
 * dispatches; the threshold is never below an ungated frame (NULL: every frame gated). */
int32_t mbls_scratch_plan(uint64_t pool_bytes, uint64_t retain_default, uint32_t queues, uint32_t cus,
                          const uint32_t* frames, const uint8_t* gated, uint32_t n_frames, mbls_scratch_plan_t* out);
/* The plan the calling thread's engine runs with (frames read from the loaded code objects,
 * queues = GPU_MAX_HW_QUEUES); MBLS_ERR_DEVICE before the engine is initialised. */
int32_t mbls_scratch_info(mbls_scratch_plan_t* out);
/* Name of the i-th kernel whose frame the engine prices (NULL past the last): the list covers
 * every kernel of libmbls that has a private segment (checked on the CPU by
 * tests/test_scratch_plan.py against the code objects' metadata). */
const char* mbls_scratch_kernel(int32_t i);
/* 1 if the engine routes every dispatch of the i-th priced kernel through the use-once gate */
int32_t mbls_scratch_kernel_gated(int32_t i);
/* The use-once gate of the calling thread's current device: out3 = {dispatches admitted, those
 * made to wait for earlier ones, largest sum of live use-once bytes admitted}. */
int32_t mbls_scratch_gate_stats(uint64_t* out3);
/* Test hook: records `code` (< 0) as engine `engine`'s failed deferred launch, as a failing
 * hipLaunchKernel in flush_verdict would.  The next synchronize of that engine (or an upload,
 * copy or free from a thread whose engine it is) returns it once; other engines' calls are not
 * affected (tests/_forced_forms_child.py scenario defer_error). */
int32_t mbls_debug_fail_deferred(int32_t engine, int32_t code);
/* Tears down every engine (streams, events, device memory, the pubkey table, the RCCL
 * communicator); the next call re-initialises.  Must not run while any call is in flight on
 * another thread.  Engine objects are never freed (a racing thread sees an engine that is not
 * ready, not freed memory); at process exit the engines are released by an atexit hook. */
void mbls_shutdown(void);
/* Human-readable message for a negative code, formatted as the reference NIF's
 * `format!("{:?}", err)` (lib.rs:22,41,55,57,69,...).  `got` is the offending length for
 * the *_LENGTH codes.  Returns the number of bytes written (excluding NUL). */
size_t mbls_status_message(int32_t code, size_t got, char* out, size_t out_len);
const char* mbls_version(void);

/* ------------------------------------------------- layer 1: `Bls` semantics -------- */
/* Each mirrors one NIF of native/bls_nif/src/lib.rs; `err_got` (may be NULL) receives the
 * offending length for *_LENGTH errors. */

/* Bls.sign/2 -> lib.rs:14-29.  out96 receives the compressed signature on MBLS_OK. */
int32_t mbls_bls_sign(mbls_bin private_key, mbls_bin message, uint8_t out96[96], size_t* err_got);

/* Bls.aggregate/1 -> lib.rs:31-51. */
int32_t mbls_bls_aggregate(const mbls_bin* signatures, size_t n, uint8_t out96[96], size_t* err_got);

/* Bls.verify/3 -> lib.rs:53-60. */
int32_t mbls_bls_verify(mbls_bin public_key, mbls_bin message, mbls_bin signature, size_t* err_got);

/* Bls.aggregate_verify/3 -> lib.rs:62-82. */
int32_t mbls_bls_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, const mbls_bin* messages,
                                  size_t n_messages, mbls_bin signature, size_t* err_got);

/* Bls.fast_aggregate_verify/3 -> lib.rs:84-100. */
int32_t mbls_bls_fast_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, mbls_bin message,
                                       mbls_bin signature, size_t* err_got);

/* Bls.eth_fast_aggregate_verify/3 -> lib.rs:102-119. */
int32_t mbls_bls_eth_fast_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, mbls_bin message,
                                           mbls_bin signature, size_t* err_got);

/* Bls.eth_aggregate_pubkeys/1 -> lib.rs:121-145.  out48 receives the compressed key. */
int32_t mbls_bls_eth_aggregate_pubkeys(const mbls_bin* public_keys, size_t n, uint8_t out48[48], size_t* err_got);

/* Flags of the fast_aggregate_verify entry points (the `eth_variant` argument):
 *  MBLS_FAV_ETH  eth_fast_aggregate_verify rules (lib.rs:102-119)
 *  MBLS_FAV_RLC  opt-in random-linear-combination batch check: one
 *                combined pairing product prod e([r_i] apk_i, H(m_i)) e(-g1, sum [r_i] sig_i)
 *                with 64-bit r_i from a per-call secret seed; if it holds, every set a pairing
 *                would decide gets {:ok, true}, otherwise every such set is verified exactly.
 *                Verdicts equal the exact ones except with probability <= 2^-64 per batch. */
#define MBLS_FAV_ETH 1
#define MBLS_FAV_RLC 2

/* Batched forms: n independent sets in ONE device submission; results[i] / err_got[i]
 * per set exactly as the single-set call would return.  Set i uses keys
 * key_off[i] .. key_off[i+1]-1 of `public_keys` (and of `messages` for aggregate_verify). */
int32_t mbls_bls_verify_batch(const mbls_bin* public_keys, const mbls_bin* messages, const mbls_bin* signatures,
                              size_t n, int32_t* results, size_t* err_got);
int32_t mbls_bls_fast_aggregate_verify_batch(const mbls_bin* public_keys, const uint32_t* key_off,
                                             const mbls_bin* messages, const mbls_bin* signatures, size_t n,
                                             int32_t eth_variant, int32_t* results, size_t* err_got);
int32_t mbls_bls_aggregate_verify_batch(const mbls_bin* public_keys, const uint32_t* key_off,
                                        const mbls_bin* messages, const uint32_t* msg_off,
                                        const mbls_bin* signatures, size_t n, int32_t* results, size_t* err_got);

/* ------------------------------------------ layer 2: device-resident batches ------- */
/* All pointers are device pointers of the selected engine's GPU (mbls_dev_select); work is
 * enqueued on `stream` (a hipStream_t, NULL = the engine's stream) and on the engine's own
 * G2 streams, and the call returns without synchronising.  Inputs are packed, fixed-size:
 * pks48[n_keys*48], msgs32[n_sets*32], sigs96[n_sets*96], sk32[n*32], key_off[n_sets+1];
 * pks48, sigs96, msgs32 and sk32 must be 16-byte aligned (hipMalloc / mbls_dev_malloc
 * allocations are).  `status` receives the per-set result code (1/0/<0).  Scratch is
 * engine-owned; calls on different caller streams that share it are ordered by the engine.
 * Completion: `status` is final once mbls_dev_synchronize(stream) returns, or on the device
 * after mbls_dev_stream_wait_engine(stream) (work or events the caller enqueues on `stream`
 * afterwards see the verdicts); mbls_dev_memcpy_d2h synchronises the engine first.  These
 * are the only ways to observe results: a long cold fast_aggregate_verify batch leaves its
 * verdict kernel unlaunched until the engine sees what follows -- another FAV / verify /
 * aggregate_verify call launches it in its throughput form (one lane per set), any other
 * engine call in its latency form (lane groups) -- so an event the caller records on `stream`
 * without mbls_dev_stream_wait_engine completes before it.  A pipelined table call
 * (mbls_dev_fast_aggregate_verify_indexed, > 1,024 sets) leaves its whole G2 side the same way:
 * signature decode, H(m) and the verdict (throughput forms when another call follows, lane
 * groups otherwise); only its table gather is enqueued by the call itself.
 * Lifetimes: inputs are read asynchronously, as by any stream-ordered API.  They may be freed
 * or overwritten through mbls_dev_free / mbls_dev_memcpy_h2d at once (both launch pending
 * verdicts and drain EVERY engine of the process first), or overwritten stream-ordered through
 * mbls_dev_memcpy_h2d_async (the copy waits on the device for all work every engine has
 * enqueued so far; no host drain); memory the caller frees or writes by other means must
 * stay untouched until the results are observed as above.  A cold call's deferred verdict
 * reads only engine-owned copies of key_off; a table call's deferred G2 side reads the caller's
 * signatures, messages, offsets and prechecks under the rules above.  `status` is written by
 * the verdict kernel, possibly after the call returned: it must stay allocated, and must not be
 * read or reused, until the results are observed (mbls_dev_free of it is safe: it drains). */
int32_t mbls_dev_fast_aggregate_verify(const uint8_t* pks48, const uint32_t* key_off, uint32_t n_keys,
                                       const uint8_t* msgs32, const uint8_t* sigs96, uint32_t n_sets,
                                       int32_t eth_variant, int32_t* status, void* stream);
int32_t mbls_dev_verify(const uint8_t* pks48, const uint8_t* msgs32, const uint8_t* sigs96, uint32_t n_sets,
                        int32_t* status, void* stream);
/* aggregate_verify: pair j of set i is (pks48[j], msgs32[j]) for key_off[i] <= j < key_off[i+1] */
int32_t mbls_dev_aggregate_verify(const uint8_t* pks48, const uint8_t* msgs32, const uint32_t* key_off,
                                  uint32_t n_pairs, const uint8_t* sigs96, uint32_t n_sets, int32_t* status,
                                  void* stream);
/* eth_aggregate_pubkeys per set: out48[n_sets*48] */
int32_t mbls_dev_aggregate_pubkeys(const uint8_t* pks48, const uint32_t* key_off, uint32_t n_keys, uint32_t n_sets,
                                   uint8_t* out48, int32_t* status, void* stream);
/* Bls.aggregate per set over device-resident signatures: set i sums sigs96[off[i] ..
 * off[i+1]-1] (NONE skipped, no group check, first undecodable signature is the error);
 * out96[n_sets*96], status MBLS_OK or the error code. */
int32_t mbls_dev_aggregate_signatures(const uint8_t* sigs96, const uint32_t* off, uint32_t n_sigs, uint32_t n_sets,
                                      uint8_t* out96, int32_t* status, void* stream);
/* validate n_keys compressed pubkeys (decompress + subgroup check); status per key
 * (0 valid, <0 error code).  Exposed for the validator-pubkey cache. */
int32_t mbls_dev_validate_pubkeys(const uint8_t* pks48, uint32_t n_keys, int32_t* status, void* stream);
/* Batched SkToPk and Sign on device buffers (key generation / signing for interop and
 * benches; secret keys must already satisfy 0 < sk < r, big-endian 32 bytes). */
int32_t mbls_dev_sk_to_pk(const uint8_t* sk32, uint32_t n, uint8_t* out48, void* stream);
int32_t mbls_dev_sign(const uint8_t* sk32, const uint8_t* msgs32, uint32_t n, uint8_t* out96, void* stream);
/* Wait for all work the engine enqueued on `stream` and on its own streams. */
int32_t mbls_dev_synchronize(void* stream);
/* Device-side join: `stream` waits for everything the engine has enqueued so far (its G2
 * streams included); an event recorded on `stream` afterwards completes with those calls. */
int32_t mbls_dev_stream_wait_engine(void* stream);

/* ------------------------------------------- batching queue ------- */
/* Thread-safe coalescing front end for single-set callers (the reference verifies one set
 * per NIF call: gossip_consumer.ex:15-18, operations.ex:52,367,470).  Each call borrows its
 * buffers, blocks, and returns exactly what the matching mbls_bls_* call returns; one worker
 * thread flushes pending calls as *_batch device submissions when max_sets are pending or
 * max_wait_us after the oldest arrived.  Calls fail with MBLS_ERR_ARGUMENT if the queue is
 * not running. */
int32_t mbls_queue_start(uint32_t max_sets, uint32_t max_wait_us);
int32_t mbls_queue_stop(void);
int32_t mbls_queue_running(void);
int32_t mbls_queue_stats(uint64_t* batches, uint64_t* sets);
int32_t mbls_queue_verify(mbls_bin public_key, mbls_bin message, mbls_bin signature, size_t* err_got);
int32_t mbls_queue_fast_aggregate_verify(const mbls_bin* public_keys, size_t n_keys, mbls_bin message,
                                         mbls_bin signature, int32_t eth_variant, size_t* err_got);

/* ------------------------------- validator pubkey table --------- */
/* The reference decompresses and KeyValidates every public key on every call
 * (native/bls_nif/src/lib.rs:92-96) after the caller gathered the committee's keys from the
 * state (lib/lambda_ethereum_consensus/state_transition/predicates.ex:122-127).  This
 * additive API keeps validated keys resident in HBM, indexed by validator index, so a FAV
 * over a committee costs one gather-and-add per key instead of ~1,560 Fp multiplications.
 * Results are those of the cold path on the same keys; a row that was never set (or an
 * index past the table) is MBLS_ERR_UNKNOWN_INDEX, ordered with the other key errors by
 * list position.  Table updates are synchronous and must not race with in-flight calls. */

/* Decode + KeyValidate n compressed keys into rows first .. first+n-1 (the table grows as
 * needed, rows in between stay unknown).  status (optional): per key 0 valid, < 0 the
 * error the cold path reports for that key.  Host buffers. */
int32_t mbls_pk_table_set(uint32_t first, const uint8_t* pks48, uint32_t n, int32_t* status);
/* the same from device buffers (status device pointer or NULL); returns when done */
int32_t mbls_dev_pk_table_set(uint32_t first, const uint8_t* pks48, uint32_t n, int32_t* status, void* stream);
uint32_t mbls_pk_table_size(void);
int32_t mbls_pk_table_clear(void);
/* fast_aggregate_verify / eth_fast_aggregate_verify of set i over table rows
 * idx[idx_off[i] .. idx_off[i+1]-1]; host buffers, per-set results as the _batch calls. */
int32_t mbls_fast_aggregate_verify_indexed_batch(const uint32_t* idx, const uint32_t* idx_off,
                                                 const mbls_bin* messages, const mbls_bin* signatures, size_t n,
                                                 int32_t eth_variant, int32_t* results, size_t* err_got);
/* device-resident form (all pointers device; asynchronous on `stream`) */
int32_t mbls_dev_fast_aggregate_verify_indexed(const uint32_t* idx, const uint32_t* idx_off, uint32_t n_idx,
                                               const uint8_t* msgs32, const uint8_t* sigs96, uint32_t n_sets,
                                               int32_t eth_variant, int32_t* status, void* stream);
/* eth_aggregate_pubkeys over table rows idx[0..n-1], host buffers: MBLS_OK and out48, or the
 * first failing row's error (MBLS_ERR_UNKNOWN_INDEX for a row never set) /
 * MBLS_ERR_EMPTY_PUBKEYS for n == 0 -- the sync-committee aggregate of accessors.ex:14-20
 * given as validator indices */
int32_t mbls_eth_aggregate_pubkeys_indexed(const uint32_t* idx, size_t n, uint8_t out48[48]);
/* eth_aggregate_pubkeys of set i over table rows (e.g. the sync committee, accessors.ex:14-20) */
int32_t mbls_dev_aggregate_pubkeys_indexed(const uint32_t* idx, const uint32_t* idx_off, uint32_t n_idx,
                                           uint32_t n_sets, uint8_t* out48, int32_t* status, void* stream);

/* -------------------------------- multi-GPU table build ------------- */
/* One process per GPU.  Verification needs no exchange (sets are independent); the only
 * collective is the optional sharded validator-table build: rank 0 makes an id
 * (mbls_comm_unique_id), the host job distributes it (e.g. torch.distributed / gloo), every
 * rank calls mbls_comm_init, then mbls_dev_pk_table_set_sharded(pks48, n, ...) with the same
 * n keys on every rank validates 1/world of them per GPU and replicates the rows with one
 * RCCL all-gather over xGMI.  status (optional, device, n) receives each key's result as
 * mbls_dev_pk_table_set would.  Without a communicator it is the local build. */
#define MBLS_COMM_ID_BYTES 128
int32_t mbls_comm_unique_id(uint8_t* out);
int32_t mbls_comm_init(const uint8_t* id, int32_t rank, int32_t world);
int32_t mbls_comm_destroy(void);
int32_t mbls_dev_pk_table_set_sharded(const uint8_t* pks48, uint32_t n, int32_t* status, void* stream);

/* ---------------------------------------- SSZ signing roots -------- */
/* The 32-byte messages the verification path consumes, computed on the device.
 * Replaces Misc.compute_signing_root/2 (state_transition/misc.ex:243-260) and the
 * Ssz.hash_tree_root/1 NIF call it makes (lib/ssz.ex:51-55) for the containers on the
 * verification path.  domain_stride: 0 = one 32-byte domain for every object, 32 = one per
 * object.  All outputs are n x 32 bytes.
 *  hash_tree_root_chunks: n fixed-size containers of `leaves` (1..16) 32-byte leaves each,
 *      packed (leaf j of object i at chunks32[(i * leaves + j) * 32]); the SSZ merkleization
 *      (zero-chunk padding to a power of two).
 *  signing_roots: hash_tree_root(SigningData{object_root, domain}).
 *  attestation_data_signing_roots: phase0 AttestationData SSZ encodings (128 bytes each)
 *      -> compute_signing_root(data, domain) (predicates.ex:118-121).
 * mbls_dev_*: device pointers, enqueued on `stream`; the plain forms take host buffers and
 * return when the roots are in `out32`. */
int32_t mbls_dev_hash_tree_root_chunks(const uint8_t* chunks32, uint32_t leaves, uint32_t n, uint8_t* out32,
                                       void* stream);
int32_t mbls_dev_signing_roots(const uint8_t* object_roots32, const uint8_t* domains32, uint32_t domain_stride,
                               uint32_t n, uint8_t* out32, void* stream);
int32_t mbls_dev_attestation_data_signing_roots(const uint8_t* data128, const uint8_t* domains32,
                                                uint32_t domain_stride, uint32_t n, uint8_t* out32, void* stream);
int32_t mbls_hash_tree_root_chunks(const uint8_t* chunks32, uint32_t leaves, size_t n, uint8_t* out32);
int32_t mbls_signing_roots(const uint8_t* object_roots32, const uint8_t* domains32, uint32_t domain_stride, size_t n,
                           uint8_t* out32);
int32_t mbls_attestation_data_signing_roots(const uint8_t* data128, const uint8_t* domains32,
                                            uint32_t domain_stride, size_t n, uint8_t* out32);

/* ------------------------------------------- device memory / stream plumbing ------- */
/* For hosts without a HIP-aware framework in the same process (the NIF, bench.py, tests):
 * thin wrappers over the HIP runtime the engine itself links. */
int32_t mbls_dev_device_count(void);
void* mbls_dev_malloc(size_t bytes);
int32_t mbls_dev_free(void* p);
int32_t mbls_dev_memcpy_h2d(void* dst, const void* src, size_t bytes);
/* enqueued on `stream` (NULL = the engine's) after all work every engine has enqueued so far;
 * returns once enqueued: `src` must stay valid until `stream` completes (pinned or not) */
int32_t mbls_dev_memcpy_h2d_async(void* dst, const void* src, size_t bytes, void* stream);
int32_t mbls_dev_memcpy_d2h(void* dst, const void* src, size_t bytes);
void* mbls_dev_stream_create(void);
int32_t mbls_dev_stream_destroy(void* stream);
void* mbls_dev_event_create(void);
int32_t mbls_dev_event_destroy(void* event);
int32_t mbls_dev_event_record(void* event, void* stream);
/* milliseconds between two recorded events (waits for `stop`); < 0 on error */
float mbls_dev_event_elapsed_ms(void* start, void* stop);

/* ------------------------------------------------------ per-kernel timing ---------- */
/* When enabled, every kernel launch of the engine is bracketed by HIP events on the stream
 * it is launched on; mbls_prof_read() resolves them and reports, for one kernel name
 * (e.g. "g1_decode_validate"), the summed duration and launch count since the last reset.
 * Names starting "path_" (path_prep_1l_table, path_prep_lg, path_prep_1l_cold,
 * path_miller_split, path_miller_joint, path_key_alt, path_verify_key_alt, path_lat_kstream2)
 * report in `launches` how many calls took that form while enabled (total_ms 0). */
int32_t mbls_prof_enable(int32_t on);
int32_t mbls_prof_reset(void);
int32_t mbls_prof_read(const char* kernel, double* total_ms, uint64_t* launches);

/* ------------------------------------------------------ batch telemetry ------------ */
/* Process-wide counters per operation, for the node's `[:bls, :batch]` telemetry events
 * (the reference has no BLS metrics, its telemetry.ex:26-85 polls VM / peer /
 * sync measurements): every API call counts once under its operation -- host batch (layer 1),
 * single-set and device-resident (layer 2) forms alike -- with the sets and public keys it
 * submitted, whether it returned an error code (< 0: argument, decode-free host errors and
 * device failures; an invalid signature is a verdict, not an error), and the wall time spent
 * inside the call (for a layer-2 call the enqueue time, its kernels run after it returns).
 * Always on: a few relaxed atomic adds per call. */
enum {
  MBLS_OP_VERIFY = 0,                /* Bls.verify */
  MBLS_OP_FAST_AGGREGATE_VERIFY,     /* Bls.fast_aggregate_verify (incl. table-indexed) */
  MBLS_OP_ETH_FAST_AGGREGATE_VERIFY, /* Bls.eth_fast_aggregate_verify (incl. table-indexed) */
  MBLS_OP_AGGREGATE_VERIFY,          /* Bls.aggregate_verify */
  MBLS_OP_ETH_AGGREGATE_PUBKEYS,     /* Bls.eth_aggregate_pubkeys (incl. table-indexed) */
  MBLS_OP_AGGREGATE,                 /* Bls.aggregate */
  MBLS_OP_SIGN,                      /* Bls.sign, SkToPk */
  MBLS_OP_KEY_VALIDATE,              /* pubkey validation, validator-table builds */
  MBLS_OP_SIGNING_ROOTS,             /* SSZ signing roots */
  MBLS_OP_COUNT
};
typedef struct mbls_op_stats {
  uint64_t calls;   /* API calls of this operation */
  uint64_t sets;    /* signature / aggregation sets (verify: 1 per pair; roots: 1 per object) */
  uint64_t keys;    /* public keys decoded or gathered */
  uint64_t errors;  /* calls that returned a negative code */
  uint64_t ns;      /* wall time inside the calls, nanoseconds */
} mbls_op_stats;
/* Operation name ("verify", "fast_aggregate_verify", ...) or NULL past MBLS_OP_COUNT. */
const char* mbls_op_name(int32_t op);
/* Copies min(n, MBLS_OP_COUNT) entries (indexed by MBLS_OP_*) into out; reset != 0 zeroes the
 * counters it copied (only those) after reading.  Returns the number of entries copied.
 * Needs no GPU. */
int32_t mbls_stats_read(mbls_op_stats* out, int32_t n, int32_t reset);

#ifdef __cplusplus
}
#endif

#endif /* MBLS_H_ */
