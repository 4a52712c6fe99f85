/*
 * hsv.h -- C ABI of the MI355X Ed25519 batch verifier (libhsv.so).
 *
 * Drop-in boundary for the reference's hot path, the `crypto` crate of
 * mwaurawakati/hotstuff-digital-signature-benchmarking:
 *
 *   crypto::Signature::verify        crypto/src/lib.rs:204-208  -> hsv_verify_strict
 *   crypto::Signature::verify_batch  crypto/src/lib.rs:210-223  -> hsv_verify_batch
 *                                                                   hsv_verify_batch_packed
 *   (batched strict API)                     -> hsv_verify
 *   crypto::Signature::new           crypto/src/lib.rs:185-191  -> hsv_sign
 *   crypto::generate_keypair         crypto/src/lib.rs:167-175  -> hsv_public_key
 *   mempool transaction check  mempool/src/batch_maker.rs:79-85 -> hsv_verify_transactions*
 *   QC / TC signature checks from wire bytes
 *                        consensus/src/messages.rs:180-198, 290-315 -> hsv_qc_verify_bincode,
 *                                                                   hsv_tc_verify_bincode
 *
 * Plain pointers and sizes only.  All inputs are borrowed for the duration of
 * the call; the library never retains a caller pointer.  Every entry point is
 * thread-safe (the reference calls verify from tokio worker threads,
 * node/src/main.rs:16).  A return value < 0 is an infrastructure error (no
 * GPU, HIP failure, bad argument) and NEVER encodes a signature rejection;
 * there is no CPU fallback for verification -- callers decide what to do.
 *
 * Byte layouts are the reference's: PublicKey = 32 bytes (crypto/src/lib.rs:66),
 * Signature = part1 (R, 32 B) || part2 (s, 32 B) as produced by flatten()
 * (lib.rs:197-202), Digest = 32 bytes (lib.rs:22).
 */
#ifndef HSV_H_
#define HSV_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Every function below is exported from libhsv.so; nothing else is (the
 * library is built with -fvisibility=hidden and a version script, and
 * tests/test_capi.py checks that its dynamic symbols are exactly these). */
#if defined(__GNUC__) || defined(__clang__)
#define HSV_API __attribute__((visibility("default")))
#else
#define HSV_API
#endif

/* ---- per-signature flag byte (hsv_verify / hsv_verify_device) ---------- */
#define HSV_STRICT_OK 0x01u /* == ed25519-dalek PublicKey::verify_strict Ok   */
#define HSV_EQ_OK 0x02u     /* PARSE_OK and [s]B == R + [k]A (cofactorless)    */
#define HSV_PARSE_OK 0x04u  /* S_OK and A_OK and R_OK                          */
#define HSV_SMALL_A 0x08u   /* A decodes and [8]A == O                         */
#define HSV_SMALL_R 0x10u   /* R decodes and [8]R == O                         */
#define HSV_S_OK 0x20u      /* s < l (canonical)                               */
#define HSV_A_OK 0x40u      /* A decompresses                                  */
#define HSV_R_OK 0x80u      /* R decompresses                                  */
/* verify_batch item accepted  <=>  (flags & (HSV_PARSE_OK|HSV_EQ_OK)) == both  */

/* ---- return codes ------------------------------------------------------- */
#define HSV_OK 0
#define HSV_ERR_NO_DEVICE (-1)
#define HSV_ERR_HIP (-2)
#define HSV_ERR_INVALID_ARG (-3)
#define HSV_ERR_ALLOC (-4)
#define HSV_ERR_ALIGN (-5)
#define HSV_ERR_PARSE (-6) /* malformed wire bytes (hsv_*_bincode) */
/* The device self-checks failed: an item's final point was not a curve point
 * (corrupted table memory, workspace or HBM) or a workspace canary changed.
 * The launch's flags are not a verdict; callers treat it like any other
 * infrastructure error (a GPU failure is never a silent reject). */
#define HSV_ERR_DEVICE_FAULT (-7)

/* ---- lifecycle and device binding -------------------------------------- */
/* Optional: contexts are created lazily on first use.
 *   device >= 0  binds the process to that GPU: every host-buffer call
 *                (hsv_verify*, hsv_verify_batch*, transactions, certificates,
 *                committee creation) runs on it.  This is the one-process-
 *                per-GPU deployment (the reference runs one node per process,
 *                node/src/main.rs:16); returns 1.
 *   device == -1 every visible GPU: host batches of >= 2^16 items are
 *                sharded across them by contiguous range (one host thread
 *                each, flags gathered into the caller's buffer); smaller
 *                batches run on the calling thread's current HIP device.
 *                Returns the number of devices.
 * Without a call, the environment variable HSV_DEVICE (same values) applies,
 * else -1.  Each device keeps a pool of HSV_SLOTS (default 4) staging slots,
 * so concurrent calls (several tokio workers) do not queue behind one buffer.
 * A slot's streams (and the device API's side streams) are created at the
 * greatest stream priority, so they draw on hardware queues of their own
 * instead of sharing the application's.
 * Device-resident calls (hsv_*_device*) always run on the device that owns
 * their input pointers; a stream of another device is an error.
 * Returns < 0 for a device index out of range. */
HSV_API int hsv_init(int device);
/* The binding in effect: a device index, or -1 for "every device". */
HSV_API int hsv_bound_device(void);
/* Release all device buffers, streams and pinned staging memory. */
HSV_API void hsv_shutdown(void);
/* Number of visible HIP devices (0 when none). */
HSV_API int hsv_device_count(void);
/* Human-readable description of the last error on the calling thread. */
HSV_API const char *hsv_last_error(void);
/* Library version string, "hsv MAJOR.MINOR.PATCH (gfx950)".  0.3.0: the
 * three device-API calls (hsv_verify_device_bits, hsv_committee_verify_device,
 * hsv_verify_transactions_device) take the optional d_fault argument before
 * `stream`; a caller built against 0.2.x headers must be rebuilt (check
 * HSV_ABI_VERSION against hsv_abi_version() at startup). */
#define HSV_ABI_VERSION 3
HSV_API const char *hsv_version(void);
/* The ABI generation this library implements (HSV_ABI_VERSION of its header). */
HSV_API int hsv_abi_version(void);

/* ---- verification, host buffers (synchronous) --------------------------- */
/* Verify n independent triples.  pk: n*32 B, sig: n*64 B (R||s),
 * msg: n*32 B when msg_stride == 32, or one shared 32-B digest when
 * msg_stride == 0 (the QC case).  flags_out: n bytes (HSV_* bits above).
 * n == 0 is valid and does nothing. */
HSV_API int hsv_verify(const uint8_t *pk, const uint8_t *sig, const uint8_t *msg, size_t msg_stride,
               size_t n, uint8_t *flags_out);

/* crypto::Signature::verify (crypto/src/lib.rs:204-208):
 * returns 1 = Ok, 0 = Err(CryptoError), < 0 = infrastructure error. */
HSV_API int hsv_verify_strict(const uint8_t digest[32], const uint8_t pk[32], const uint8_t sig[64]);

/* crypto::Signature::verify_batch (crypto/src/lib.rs:210-223), votes as
 * parallel arrays pk[n*32], sig[n*64] over one shared digest:
 * returns 1 = Ok, 0 = Err, < 0 = infrastructure error.  n == 0 -> 1 (Ok). */
HSV_API int hsv_verify_batch(const uint8_t digest[32], const uint8_t *pk, const uint8_t *sig, size_t n);

/* Same, votes packed as n 96-byte records pk(32)||R(32)||s(32). */
HSV_API int hsv_verify_batch_packed(const uint8_t digest[32], const uint8_t *votes, size_t n);

/* Automatic committee cache behind hsv_verify_batch[_packed] (on by default;
 * env HSV_AUTO_COMMITTEE=0 turns it off).  Consensus keys repeat every round
 * (consensus/src/config.rs Committee): a key seen in two batches is queued,
 * and a background thread builds its comb table on a stream of its own and
 * appends it to the cache (at most 8192 keys, 384 KiB each; batches of more
 * than 8192 votes are never cached).  A verify call never waits for a build:
 * batches whose keys are all cached take the committee kernels, all others
 * the generic kernels, with identical flags either way.  A failed build is a
 * cache miss, never an error; when a full cache keeps missing (a new epoch)
 * it is dropped and relearnt.  Strict batches of <= 4096 cached keys
 * (hsv_verify, hsv_verify_strict) use it too.  enable = 0 also drops it. */
HSV_API int hsv_set_auto_committee(int enable);
/* Number of keys in the automatic cache (0 when none). */
HSV_API size_t hsv_auto_committee_size(void);
/* Wait up to timeout_ms for a pending cache build to be published:
 * 1 = no build in flight, 0 = timed out.  (Warm-up and tests.) */
HSV_API int hsv_auto_committee_wait(int timeout_ms);
/* Number of cached-path launches whose device self-check failed since the
 * process started.  Such a call is answered by the generic kernels instead,
 * and the cache is dropped and relearnt (its tables are no longer trusted). */
HSV_API uint64_t hsv_auto_committee_faults(void);

/* Resident latency service (on by default; env HSV_QC_RESIDENT=0 turns it
 * off).  Calls of 1-4 votes whose keys are all in a committee cache
 * (hsv_verify_strict, small hsv_verify / hsv_verify_batch*, the explicit
 * committee) are posted to one block of the latency kernel that stays on a CU
 * of the home device, instead of a launch each: one verify_strict costs
 * about 0.034 ms instead of 0.039 ms.  The block leaves after
 * HSV_QC_RESIDENT_IDLE_MS (default 50) without a request and is relaunched by
 * the next one; while it runs it holds one CU, so a device-wide
 * synchronisation of the application (hipDeviceSynchronize) waits at most
 * that idle time.  The library pauses it around its own frees, and its
 * persistent large-batch grids leave one CU free once it has run.  Verdicts
 * never depend on it: a request it does not answer goes to the launch path.
 * mode 1 = on, 0 = off (the block stops before the call returns).  Returns
 * the previous mode. */
HSV_API int hsv_set_resident_service(int mode);

/* ---- verification, device-resident buffers (stream-ordered, async) ------ */
/* Inputs already in HBM (of any device: the call runs on the device owning
 * d_pk, and `stream` must belong to it).  Record i reads
 * pk + i*pk_stride (32 B), sig + i*sig_stride (64 B), msg + i*msg_stride
 * (32 B; msg_stride may be 0).  Pointers and strides must be multiples of 16.
 * Writes n flag bytes to d_flags.  stream: a hipStream_t (NULL = default).
 * Does not synchronise.  Batches above 2^22 items run as 2^22-item launches
 * alternating over `stream` and a library stream forked from and joined back
 * into `stream` by events: the call stays ordered on `stream` as one unit. */
HSV_API int hsv_verify_device(const uint8_t *d_pk, size_t pk_stride, const uint8_t *d_sig,
                      size_t sig_stride, const uint8_t *d_msg, size_t msg_stride, size_t n,
                      uint8_t *d_flags, void *stream);

/* As hsv_verify_device, additionally packing STRICT_OK bits into
 * d_strict_bits[(n+31)/32] (bit i of word i/32 = item i).  Either output
 * pointer may be NULL.
 * d_fault (optional): two device words owned by the caller.  The library
 * zeroes them on `stream` before the call's launches and the kernels set
 * d_fault[0] (a final point failed the curve self-check) and d_fault[1] (a
 * workspace canary changed, i.e. memory the launch wrote was overwritten).
 * Read them after synchronising `stream`: both zero means the flags are a
 * verdict, anything else is an infrastructure error (HSV_ERR_DEVICE_FAULT on
 * the host-buffer calls).  The words belong to this call alone, so concurrent
 * callers on other streams never see or clear each other's faults.  With
 * d_fault NULL the launches report into the per-device word read by
 * hsv_device_faults. */
HSV_API int hsv_verify_device_bits(const uint8_t *d_pk, size_t pk_stride, const uint8_t *d_sig,
                           size_t sig_stride, const uint8_t *d_msg, size_t msg_stride, size_t n,
                           uint8_t *d_flags, uint32_t *d_strict_bits, uint32_t *d_fault, void *stream);

/* Self-check results of the device-resident calls on `device` (-1: every
 * device) that ran without a d_fault of their own, since the last clear.
 * Read after synchronising the streams those calls ran on.  Returns 0 (no
 * fault), the fault bits (1: curve check, 2: canary), or < 0 on error.
 * clear != 0 reads and resets the word in one atomic exchange on the device,
 * so a fault recorded by a launch still running on another stream is either
 * returned now or kept for the next read, never lost.  Host-buffer calls
 * report their own launches' faults as HSV_ERR_DEVICE_FAULT instead. */
HSV_API int hsv_device_faults(int device, int clear);

/* ---- committee key cache --------------------------- */
/* Consensus keys are fixed per epoch (consensus/src/config.rs Committee).  A
 * committee holds, in HBM of the device bound at creation (hsv_init), a 384 KiB
 * fixed-base comb table of -A per key; verifying a vote by a member then costs
 * 64 mixed additions and no doublings.  Flags are identical to hsv_verify's
 * (undecodable or small-order keys are accepted as members and reported
 * through HSV_A_OK / HSV_SMALL_A exactly as the generic path does). */
typedef struct hsv_committee hsv_committee;
/* Build tables for n public keys (n*32 B). */
HSV_API int hsv_committee_create(const uint8_t *pks, size_t n, hsv_committee **out);
HSV_API void hsv_committee_destroy(hsv_committee *c);
HSV_API size_t hsv_committee_size(const hsv_committee *c);
/* Index of pk in the committee, or -1. */
HSV_API int64_t hsv_committee_index(const hsv_committee *c, const uint8_t pk[32]);
/* Votes by member index: key_idx[m], sig m*64 B, msg m*32 B (msg_stride 32)
 * or one shared digest (msg_stride 0); flags_out m bytes.  An index >= n
 * yields flags 0. */
HSV_API int hsv_committee_verify(hsv_committee *c, const uint32_t *key_idx, const uint8_t *sig,
                         const uint8_t *msg, size_t msg_stride, size_t m, uint8_t *flags_out);
/* crypto::Signature::verify_batch over votes packed pk||R||s: members use the
 * cached tables, any other key the generic kernel.  1 = Ok, 0 = Err, < 0 error. */
HSV_API int hsv_committee_verify_batch_packed(hsv_committee *c, const uint8_t digest[32], const uint8_t *votes,
                                      size_t m);
/* Device-resident, stream-ordered form (device = the committee's); d_fault
 * (optional) as hsv_verify_device_bits. */
HSV_API int hsv_committee_verify_device(const hsv_committee *c, const uint32_t *d_key_idx, const uint8_t *d_sig,
                                size_t sig_stride, const uint8_t *d_msg, size_t msg_stride, size_t m,
                                uint8_t *d_flags, uint32_t *d_fault, void *stream);

/* ---- mempool transactions -------------------------- */
/* A client transaction is  message || pk (32 B) || sig (64 B, R||s)  and its
 * signature is checked over Digest(SHA-512(message)[..32]) with
 * Signature::verify, as in the reference's transaction check
 * (mempool/src/batch_maker.rs:79-85, consensus/src/core.rs:121-127).  The
 * per-transaction flags are hsv_verify's flags for that (pk, sig, digest);
 * HSV_STRICT_OK is the reference's `signature.verify(..).is_ok()`.
 * Transactions shorter than 96 bytes (the reference's slice would panic) are
 * rejected with HSV_ERR_INVALID_ARG by the host-buffer calls. */

/* Ragged batch: transaction i is txs[offsets[i] .. offsets[i+1]) (n+1
 * offsets).  flags_out: n bytes. */
HSV_API int hsv_verify_transactions(const uint8_t *txs, const uint64_t *offsets, size_t n, uint8_t *flags_out);

/* Fixed-size batch (the benchmark client's transactions all have the same
 * size, node/src/client.rs): transaction i is txs[i*tx_size .. (i+1)*tx_size). */
HSV_API int hsv_verify_transactions_fixed(const uint8_t *txs, size_t tx_size, size_t n, uint8_t *flags_out);

/* Device-resident, stream-ordered form.  d_offsets (n+1 entries, relative to
 * d_txs) or NULL for fixed-size transactions of tx_size bytes.  Any alignment
 * of d_txs.  Transactions shorter than 96 bytes get flags 0.  Outputs and
 * d_fault as hsv_verify_device_bits (d_flags / d_strict_bits: either may be
 * NULL, not both). */
HSV_API int hsv_verify_transactions_device(const uint8_t *d_txs, const uint64_t *d_offsets, size_t tx_size, size_t n,
                                   uint8_t *d_flags, uint32_t *d_strict_bits, uint32_t *d_fault, void *stream);

/* ---- wire formats ---------------------------------- */
/* Certificates verified straight from their bincode bytes (bincode 1.3
 * defaults: little-endian, u64 lengths; PublicKey is its base64 string,
 * crypto/src/lib.rs:94-101).  Only the signature part of the reference's
 * verify is done here; the quorum/stake checks stay with the caller, who can
 * get the decoded keys back.  Returns 1 = Ok, 0 = Err (a signature fails),
 * HSV_ERR_PARSE for malformed bytes, other < 0 for infrastructure errors. */

/* consensus::QC (consensus/src/messages.rs:162-167): hash (32) | round (u64)
 * | votes Vec<(PublicKey, Signature)>.  Checks
 * Signature::verify_batch(&qc.digest(), &qc.votes) (messages.rs:196-197),
 * qc.digest() = SHA-512(hash || round_le)[..32] (messages.rs:201-207).
 * n_votes_out (optional): number of votes; pks_out (optional, 32 B per vote):
 * the decoded keys, in order. */
HSV_API int hsv_qc_verify_bincode(const uint8_t *buf, size_t len, size_t *n_votes_out, uint8_t *pks_out);

/* consensus::TC (messages.rs:281-285): round (u64) | votes
 * Vec<(PublicKey, Signature, Round)>.  Checks every vote with
 * Signature::verify over SHA-512(round_le || high_qc_round_le)[..32]
 * (messages.rs:306-313); 1 iff all pass.  flags_out (optional, one byte per
 * vote): the per-vote HSV_* flags. */
HSV_API int hsv_tc_verify_bincode(const uint8_t *buf, size_t len, size_t *n_votes_out, uint8_t *flags_out);

/* ---- signing (host CPU; not on the hot path) ---------------------------- */
/* Public key for a 32-byte secret seed (dalek Keypair from SecretKey). */
HSV_API int hsv_public_key(const uint8_t seed[32], uint8_t pk_out[32]);
/* RFC 8032 deterministic signature (Signature::new). */
HSV_API int hsv_sign(const uint8_t seed[32], const uint8_t *msg, size_t msg_len, uint8_t sig_out[64]);
/* Bulk: n seeds (n*32 B), n messages of msg_len bytes each; writes n public
 * keys and n signatures.  nthreads <= 0 picks min(hardware concurrency, 16). */
HSV_API int hsv_sign_many(const uint8_t *seeds, const uint8_t *msgs, size_t msg_len, size_t n,
                  uint8_t *pk_out, uint8_t *sig_out, int nthreads);

/* Synthesis helper for the corrupted-input mixes (SURVEY 8(d) C3/C4 "mixed-
 * order A"; Appendix A.3 rows 7-8): the key A' = [a]B + [2*torsion+1]T8 (a
 * from seed as in hsv_public_key, T8 a point of order 8, torsion in 0..3) and
 * a signature over msg whose challenge k is = 0 (mod 8) when accept != 0
 * (verify_strict accepts: cofactorless equation holds) or != 0 (mod 8) when
 * accept == 0 (rejected; a cofactored verifier would accept). */
HSV_API int hsv_sign_mixed_order(const uint8_t seed[32], const uint8_t *msg, size_t msg_len, int torsion, int accept,
                         uint8_t pk_out[32], uint8_t sig_out[64]);

/* ---- measurement helpers ------------------------------------------------ */
/* Measured issue rate of v_mad_u64_u32 on the current device, in
 * multiply-accumulates per second (the roofline denominator). */
HSV_API double hsv_measure_mad_peak(void);
/* Kernel variant id the library runs (21: the product default). */
HSV_API int hsv_get_variant(void);
/* Host threads of the staging-copy pool, the calling thread excluded. */
HSV_API int hsv_pack_threads(void);
/* The calling thread's last host-buffer verification: host milliseconds spent
 * packing into pinned staging, bytes copied host-to-device, wall milliseconds
 * of the call (any pointer may be NULL). */
HSV_API void hsv_host_call_stats(double *pack_ms, double *h2d_bytes, double *call_ms);
/* Host timeline of the calling thread's last call, milliseconds from its
 * entry.  For a latency call (one launch: a QC, a vote, a small batch) the
 * HSV_MARK_* points below (a point the call did not pass reads -1); for a
 * pipelined call four marks per chunk (staging buffer free, packed, copy
 * enqueued, launch enqueued).  Writes min(count, cap) values to out (may be
 * NULL) and returns the count. */
#define HSV_MARK_LOOKUP 0  /* committee-cache lookup done                 */
#define HSV_MARK_SLOT 1    /* staging slot leased                         */
#define HSV_MARK_STAGED 2  /* inputs packed into pinned staging           */
#define HSV_MARK_LAUNCH 3  /* kernel launch enqueued                      */
#define HSV_MARK_SYNC 4    /* stream synchronisation returned             */
#define HSV_MARK_DONE 5    /* flags copied out, self-check words read     */
#define HSV_MARKS 6
HSV_API int hsv_host_call_marks(double *out, int cap);

#ifdef __cplusplus
}
#endif

#endif /* HSV_H_ */
