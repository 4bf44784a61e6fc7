/*
 * dpwa_hip.h -- C ABI of libdpwa_hip.so, the MI355X-native pairwise-averaging hot path.
 *
 * The reference (zenghanfu/dpwa) is pure Python; its hot path is the adapter/connection
 * seam below, which this library replaces.  Every entry point names the reference
 * interface it stands in for.  A maintainer binds it with ctypes;
 * dpwa_amd/_lib.py is that binding.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Device pointers are HIP device addresses on the
 *    learner's GPU; `dpwa_stream_t` is a hipStream_t (NULL = the legacy default stream).
 *  - Every function returns DPWA_OK (0) or a negative DPWA_ERR_*; the message of the
 *    last failure on the calling thread is available from dpwa_last_error().
 *  - The library never allocates or frees caller memory.  Learner-owned snapshot and
 *    staging buffers are allocated at dpwa_learner_create() with hipMalloc.
 *  - No host synchronisation happens inside publish / fetch / average: the factor is
 *    computed on the device from the (clock, loss) state and handed to the lerp through
 *    device memory (dpwa_coef), so a whole round can be enqueued without a sync.
 *  - There is no CPU fallback: without a HIP device the compute entry points fail.
 */
#ifndef DPWA_HIP_H
#define DPWA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPWA_ABI_VERSION 10

#define DPWA_OK 0
#define DPWA_ERR_ARG (-1)     /* bad argument (API misuse)                          */
#define DPWA_ERR_HIP (-2)     /* a HIP runtime call failed                          */
#define DPWA_ERR_STATE (-3)   /* call out of order (e.g. average without a fetch)   */
#define DPWA_ERR_NOMEM (-4)

/* element types of the flat parameter buffer */
#define DPWA_F32 0            /* the reference's only type: TYPE_CONVERSION, pytorch.py:11-14 */
#define DPWA_BF16 1           /* extension: torch-eager bf16 rounding, no reference path      */
#define DPWA_F64 2            /* loss scalars only (dpwa_learner_set_loss_dtype)              */

/* interpolation methods: INTERPOLATION_METHODS, dpwa/dpwa.py:11-15 */
#define DPWA_INTERP_CONSTANT 0   /* interpolation.py:8-15  factor = value                       */
#define DPWA_INTERP_CLOCK 1      /* interpolation.py:18-24 factor = peer_clock/(clock+peer_clock) */
#define DPWA_INTERP_LOSS 2       /* interpolation.py:27-33 factor = loss/(loss+peer_loss)         */

/* status written into dpwa_coef.status by the factor kernel */
#define DPWA_STATUS_OK 0
#define DPWA_STATUS_ZERO_DIVISION 1   /* the reference raises ZeroDivisionError (dpwa.py:143) */

typedef void *dpwa_stream_t;

/* The published `state` of one learner (dpwa.py:115 `{'clock', 'loss'}`), stored as the
 * first 256 bytes of every snapshot slot so that state and parameters travel together
 * exactly as RxThread sends them together (conn.py:110). */
/* A snapshot slot is [dpwa_header | zero pad | payload]: the payload starts 4 KiB into the
 * slot, so every 1-KiB wave span of the averaging kernel lies inside one aligned 1-KiB block
 * (a payload right behind the 256-B header made each span straddle two: 0.7 % slower at
 * 11.17M fp32 and 2 % at 100M, tools/skew_tune.hip). */
#define DPWA_SLOT_PAYLOAD_OFFSET 4096
typedef struct dpwa_header {
    double clock;        /* publisher's clock after `clock += 1` (dpwa.py:112)           */
    double loss;         /* loss given to update_send (dpwa.py:115)                      */
    uint64_t version;    /* publishes so far; 0 = never published (have_state, conn.py:60) */
    int64_t n;           /* payload elements                                              */
    int32_t dtype;       /* DPWA_F32 / DPWA_BF16                                          */
    int32_t reserved0;
    uint8_t pad[216];
} dpwa_header;

/* Averaging coefficients, produced on the device by the factor kernel (dpwa.py:143-150)
 * and consumed by the lerp (pytorch.py:68). */
typedef struct dpwa_coef {
    double factor;       /* interpolation factor after divergence scaling (dpwa.py:143-147) */
    double new_clock;    /* factor*peer_clock + (1-factor)*clock (dpwa.py:150)              */
    float a;             /* f32(factor)        -- torch casts the scalar to fp32            */
    float b;             /* f32(1.0 - factor)  -- `1 - factor` is a Python double           */
    int32_t status;      /* DPWA_STATUS_*; non-zero makes the lerp a no-op                  */
    int32_t reserved;
} dpwa_coef;

/* Interpolation configuration (DpwaConfiguration.get_interpolation / get_divergence_threshold,
 * dpwa.py:40-51). */
typedef struct dpwa_interp {
    int32_t method;               /* DPWA_INTERP_*                                 */
    int32_t reserved;
    double value;                 /* constant value (ConstantInterpolation)        */
    double divergence_threshold;  /* 0 disables (README.md:62)                     */
} dpwa_interp;

const char *dpwa_last_error(void);
int dpwa_abi_version(void);

/* roctx ranges on the round (the reference's LOGGER.debug sites dpwa.py:119,152-153,
 * conn.py:242-243,296).  On only when DPWA_ROCTX=1 is set when the library loads: then
 * dpwa.update_send / dpwa.publish / dpwa.fetch_loop / dpwa.update_wait_average / dpwa.average
 * (and the learner's publish) are pushed as ranges that `rocprofv3 --marker-trace` records.
 * dpwa_trace_push/pop let the layer above add its own (no-ops when off).  ABI version 8. */
int dpwa_trace_enabled(void);
int dpwa_trace_push(const char *name);
int dpwa_trace_pop(void);

/* Last words (bench.py's held result line): registers `line` (len bytes, at most 16 KiB; len 0
 * clears it) to be written to `fd` with write(2) if the process is ended by SIGTERM, SIGINT,
 * SIGHUP, SIGABRT, SIGSEGV, SIGBUS, SIGFPE or SIGILL; the handler then restores the previous
 * handler and re-raises.  The first call installs the handlers.  dpwa_last_words_flush writes
 * the registered line now; the line is written at most once, by the flush or by a signal,
 * whichever claims it first (*wrote = 1 when the flush did).  ABI version 10. */
int dpwa_last_words_set(int fd, const char *line, int64_t len);
int dpwa_last_words_flush(int *wrote);
int dpwa_last_words_written(int *written);

/* ------------------------------------------------------------------------------------
 * Stateless kernels (the fused replacements of the ATen mul/mul/add behind pytorch.py:68)
 * ------------------------------------------------------------------------------------ */

/* param[i] = f32(f32(a*peer[i]) + f32(b*param[i])) with (a, b) read from coef_dev on the
 * device (no host sync).  Replaces the per-tensor loop dpwa/adapters/pytorch.py:66-68 with
 * one launch over the flat buffer.  In place; param and peer may not overlap. */
int dpwa_lerp_f32(float *param, const float *peer, int64_t n, const dpwa_coef *coef_dev,
                  dpwa_stream_t stream);
/* bf16 form: bf16(bf16(a*peer) + bf16(b*param)), RNE (torch-eager bf16). */
int dpwa_lerp_bf16(uint16_t *param, const uint16_t *peer, int64_t n, const dpwa_coef *coef_dev,
                   dpwa_stream_t stream);
/* Same kernels with the factor given by the host, as pytorch.py:68 receives it. */
int dpwa_lerp_f32_host(float *param, const float *peer, int64_t n, double factor, dpwa_stream_t stream);
int dpwa_lerp_bf16_host(uint16_t *param, const uint16_t *peer, int64_t n, double factor,
                        dpwa_stream_t stream);

/* The fused average of dpwa_learner_average without a learner (the product kernel over
 * caller-owned buffers): reads clock_dev[0] and the 256-B dpwa_header at `peer_slot`, lerps the
 * n elements at peer_slot + DPWA_SLOT_PAYLOAD_OFFSET into `param` in place, writes clock_dev[1] = new clock and
 * *coef_dev.  snap_payload (NULL or n elements): the write-through form, which also stores the
 * result there (dpwa_learner_average_through).  start_event/stop_event (hipEvent_t, both or neither): the kernel is launched with
 * hipExtLaunchKernelGGL so they record its own begin and end (measurement). */
int dpwa_average(int32_t dtype, void *param, const void *peer_slot, int64_t n, const dpwa_interp *cfg,
                 double *clock_dev, double loss, dpwa_coef *coef_dev, void *snap_payload, dpwa_stream_t stream,
                 void *start_event, void *stop_event);

/* dpwa_average over several independent (param, peer slot) pairs in ONE dispatch -- the averages
 * of co-resident learners of one round (pytorch.py:66-68 once per learner).  Each descriptor is
 * one dpwa_average call: its own clock_dev (reads [0], writes [1]), coefficient block and loss;
 * all share `cfg` and `dtype`, and either all or none write through (snap_payload).  Every
 * pointer 16-B aligned; 1..8 descriptors.  Events as dpwa_average (the whole dispatch). */
typedef struct dpwa_average_desc {
    void *param;
    const void *peer_slot;   /* [dpwa_header | pad | payload] */
    int64_t n;
    double *clock_dev;
    double loss;
    dpwa_coef *coef_dev;
    void *snap_payload;      /* NULL, or n elements: the write-through destination */
} dpwa_average_desc;
int dpwa_average_many(int32_t dtype, const dpwa_average_desc *descs, int count, const dpwa_interp *cfg,
                      dpwa_stream_t stream, void *start_event, void *stop_event);
/* The same in the resident form (dpwa_learner_set_resident below): each `param` is read only and the
 * result goes to its snap_payload (required for n > 0) -- 3*n*s bytes per descriptor.  One
 * descriptor runs the single-learner kernel, several the batched one.  Equal-size descriptors whose
 * reads overlap (a `param` is another descriptor's peer payload, or two share a peer: co-resident
 * learners that picked each other, e.g. a mutual pair) run one fused pass that reads each distinct
 * buffer once, up to 8 of them; beyond that the repeated reads are dispatched to hit L2. */
int dpwa_average_many_resident(int32_t dtype, const dpwa_average_desc *descs, int count, const dpwa_interp *cfg,
                               dpwa_stream_t stream, void *start_event, void *stop_event);

/* Factor + clock on the device (dpwa.py:139-155 + interpolation.py): reads *clock_dev and the
 * peer's header, writes *coef_dev and, unless the status is an error, *clock_dev = new_clock.
 * `loss` is used when loss_dev is NULL, else *loss_dev (a device float64). */
int dpwa_factor(const dpwa_interp *cfg, double *clock_dev, const dpwa_header *peer_header_dev, double loss,
                const double *loss_dev, dpwa_coef *coef_dev, dpwa_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Learner runtime: one per gossip node.  Owns two snapshot slots (double-buffered
 * RxThread.set_current_state, conn.py:73-79), a staging buffer (the fetched
 * TxThread.peer_payload, conn.py:298), the device clock and the coefficient block.
 * ------------------------------------------------------------------------------------ */
typedef struct dpwa_learner dpwa_learner;

int dpwa_learner_create(dpwa_learner **out, int device, int64_t n, int32_t dtype, const dpwa_interp *cfg);

/* Measurement only (bench.py `roofline.mix_ceiling`; no reference interface): the averaging
 * kernels' access mix with nothing else in it -- every 1-KiB span of `nr` (1-2) source buffers
 * loaded and one sum of them stored into `nw` (1-2) destinations, `nbytes` (a multiple of 16)
 * each, with the product kernel's launch shape and cache policy.  nr = 2, nw = 2 is the
 * write-through average's mix (read parameters and snapshot, write parameters and next
 * snapshot).  start/stop: optional dispatch begin/end events. */
int dpwa_stream_mix(void *const *dst, int nw, const void *const *src, int nr, int64_t nbytes, dpwa_stream_t stream,
                    void *start_event, void *stop_event);
int dpwa_learner_destroy(dpwa_learner *l);

/* update_send's publish half (dpwa.py:111-116 + pytorch.py:49-53): clock += 1 on the device,
 * copy the n-element flat buffer into the next snapshot slot with header {clock, loss,
 * version}.  Stream-ordered after prior work on `stream`. */
int dpwa_learner_publish(dpwa_learner *l, const void *flat, double loss, const double *loss_dev,
                         dpwa_stream_t stream);
/* Number of publishes so far (host counter, no sync). */
int dpwa_learner_version(const dpwa_learner *l, uint64_t *version);

/* Peers.  `peer_id` is the caller's index of that peer (e.g. its node index).
 * attach_local: the peer learner lives in this process (any device); peer == l is the
 * self-peer (a YAML node at the learner's own host:port: its own published snapshot).
 * ipc_handle / attach_ipc: the peer lives in another process; ipc_handle describes the
 * snapshot allocation (handle_len = DPWA_IPC_HANDLE_BYTES) and, for an ordinary allocation,
 * carries its hipIpcGetMemHandle.  Allocations of 1.5 GiB and more (or any size with
 * DPWA_VMM=1) are hipMemCreate chunks instead -- hipIpcOpenMemHandle does not return for
 * allocations above ~2 GiB on this ROCm stack -- and are shared as POSIX fds:
 * export_fds (which = 0: snapshot slots, 1: relay buffer) yields one fd per chunk, *n_fds = 0
 * for an ordinary allocation; the caller passes them to the peer process (e.g. SCM_RIGHTS over
 * a Unix socket) and closes its copies; the peer maps them with attach_fds (the fds stay the
 * caller's). */
#define DPWA_IPC_HANDLE_BYTES 128
int dpwa_learner_attach_local(dpwa_learner *l, int peer_id, dpwa_learner *peer);
int dpwa_learner_ipc_handle(dpwa_learner *l, void *handle_out, int64_t handle_len);
int dpwa_learner_attach_ipc(dpwa_learner *l, int peer_id, const void *handle, int64_t handle_len);
int dpwa_learner_export_fds(dpwa_learner *l, int which, int *fds, int max_fds, int *n_fds, int64_t *chunk_bytes);
int dpwa_learner_attach_fds(dpwa_learner *l, int peer_id, const void *handle, int64_t handle_len, const int *fds,
                            int n_fds, int64_t chunk_bytes);

/* The fetch (TxThread request -> reply, conn.py:297-298): pull peer `peer_id`'s snapshot of
 * publish number `peer_version` (1-based) into this learner's staging buffer on the
 * learner's side stream, after all work already enqueued on `stream`.  flags:
 * DPWA_FETCH_ZERO_COPY -- for a peer on the same device no bytes move: the average reads the
 * peer's slot in place; DPWA_FETCH_PUBLISHED -- an IPC peer's snapshot whose publish is
 * already complete (the gossip board advertised it): the pull is not ordered after `stream`
 * and alternates between two staging buffers, waiting only for the average that last read
 * the one it fills.  Slot reuse is protected for local peers by events; for IPC peers by the
 * caller's lock-step barrier or the board's read marks. */
#define DPWA_FETCH_ZERO_COPY 1
#define DPWA_FETCH_PUBLISHED 2
/* DPWA_FETCH_RESCUE: the fetch re-selected after a timed-out pull (conn.py:304-309 reconnects and
 * picks again): it copies into a rescue lane -- a buffer and a stream of the greatest priority of
 * its own -- so the stalled pull ahead of it on the side stream cannot hold it up.  A lane whose
 * pull has not landed stays taken and the next re-selected pull takes another (lanes made at first
 * use, up to 8, see rescue_free); DPWA_ERR_STATE when no lane is free. */
#define DPWA_FETCH_RESCUE 4
int dpwa_learner_fetch(dpwa_learner *l, int peer_id, uint64_t peer_version, int flags,
                       dpwa_stream_t stream);
/* The fetch timeout of the device path (the reference's socket timeout, conn.py:249 with
 * timeout_ms from the YAML, and its handling at conn.py:304-309).  fetch_state polls the copying
 * fetch in flight without blocking: DPWA_FETCH_LANDED (landed, or nothing to wait for),
 * DPWA_FETCH_IN_FLIGHT, or DPWA_FETCH_TIMED_OUT (still in flight timeout_ms after the request went
 * out).  The reference's socket timeout bounds only the wait for the reply (conn.py:249), so a pull
 * ordered after the caller's stream (a local peer's snapshot) is timed from when that stream
 * reached update_send -- a device backlog the caller queued before update_send is not the peer's
 * delay: while the stream has not reached it the pull is in flight, after it the time since is read
 * on the device's clock (an event on a probe stream of its own, timestamps compared); a backlog of
 * over 60 s, or a probe that cannot run, falls back to the host's issue time.  Board pulls wait
 * for nothing of the caller's and are timed from the issue.  Judged pulls are LocalGroup copying
 * pulls and board pulls.  rescue_free: *free_out = 1 when a rescue lane is free (its pull landed) or one
 * could be made now (it is made here: up to 8 lanes, each one snapshot, while 1 GiB stays free on
 * the device; a failed allocation caps the count where it is, *free_out = 0, no error).
 * rescue_lanes: lanes made so far and the current cap; set_rescue_cap lowers (or raises, up to 8)
 * the cap -- not below the lanes already made.  fetch_stream: the stream the fetch in flight moves
 * its bytes on (side stream or a rescue lane's). */
#define DPWA_FETCH_LANDED 0
#define DPWA_FETCH_IN_FLIGHT 1
#define DPWA_FETCH_TIMED_OUT 2
int dpwa_learner_fetch_state(dpwa_learner *l, int64_t timeout_ms, int *state);
int dpwa_learner_rescue_free(dpwa_learner *l, int *free_out);
int dpwa_learner_rescue_lanes(dpwa_learner *l, int *lanes, int *cap);
int dpwa_learner_set_rescue_cap(dpwa_learner *l, int cap);
int dpwa_learner_fetch_stream(dpwa_learner *l, dpwa_stream_t *stream);

/* update_wait's averaging (dpwa.py:133-155 + pytorch.py:64-68) as ONE kernel: make `stream`
 * wait for the fetch, then every workgroup evaluates the factor (fp64, from the device clock
 * and the peer's header) while its loads are in flight and lerps its part of the n-element
 * flat buffer in place; workgroup 0 writes the new clock and the dpwa_coef. */
int dpwa_learner_average(dpwa_learner *l, void *flat, double loss, const double *loss_dev,
                         dpwa_stream_t stream);

/* Write-through form: the averaged parameters are also stored into the slot of the NEXT
 * publish (4*n*s bytes instead of 3*n*s here, and that publish then moves no payload). */
int dpwa_learner_average_through(dpwa_learner *l, void *flat, double loss, const double *loss_dev,
                                 dpwa_stream_t stream);
/* The averages of `count` learners of one device (each with a fetch in flight) as few
 * dispatches as possible: every learner's dpwa_learner_average(_through) (write_through[i]),
 * same results and bookkeeping, but compatible ones (same dtype and form, 16-B aligned,
 * contiguous source) share one launch of up to 8.  loss_dev may be NULL (all host losses). */
int dpwa_learner_average_many(dpwa_learner *const *learners, void *const *flats, const double *loss,
                              const double *const *loss_dev, const int *write_through, int count,
                              dpwa_stream_t stream);
/* always != 0: a write-through average never writes the next publish's header ahead; that
 * publish then writes it with the loss given to it (a snapshot served over the wire bridge
 * carries the reference's {'clock', 'loss'} state, conn.py:110). */
int dpwa_learner_set_header_publish(dpwa_learner *l, int always);
/* Publish that reuses a write-through snapshot when the last average wrote `flat` through
 * (the caller asserts `flat` is unchanged since): header only; otherwise a full publish. */
int dpwa_learner_publish_reuse(dpwa_learner *l, const void *flat, double loss, const double *loss_dev,
                               dpwa_stream_t stream);
/* on != 0: a reusing publish (above) first compares 4096 16-B words spread over `flat` with
 * the written-through snapshot on the device, and copies the payload from `flat` when any
 * differs -- a write the caller's bookkeeping missed (pytorch.py:49-53 then holds anyway: the
 * snapshot is the parameters at update_send).  Two small launches, no host sync.
 * reuse_guard_hits: how many publishes found a difference (synchronises the device).
 * On a resident learner (below) the same flag is the window guard: every publish runs one small
 * kernel that compares the payload published last time with those words saved when it was
 * published -- a write while peers could read it (update_send .. update_wait, through
 * `param.data`, which the adapter's version counters miss) -- and saves the new payload's.  A
 * written window is reported by the first publish that finds it counted (never waiting for a
 * check): DPWA_ERR_STATE, nothing published; the publish after proceeds.  window_hits: windows
 * found written so far, checking the last one now (synchronises its stream). */
int dpwa_learner_set_reuse_guard(dpwa_learner *l, int on);
int dpwa_learner_reuse_guard_hits(dpwa_learner *l, uint32_t *hits);
int dpwa_learner_window_hits(dpwa_learner *l, uint32_t *hits);

/* Resident parameters (extension; replaces the snapshot copy of pytorch.py:49-53 and
 * RxThread.set_current_state, conn.py:73-79, with no copy at all).  The learner's parameters live
 * in its own two snapshot slots and move between them: a publish writes only the header of the
 * slot they are in, and the average reads them there -- the published snapshot, which it leaves
 * untouched -- and stores the result into the other slot, the slot of the next publish.  A round
 * then moves 3*n*s bytes, the averaging's own (write-through: 4*n*s; publish + in-place average:
 * 5*n*s), with the same results.
 *   set_resident      before the first publish: copy `init` (n elements) into slot 0.
 *   resident_params   where the parameters are now (*params NULL and *slot -1 when not resident):
 *                     a device pointer valid for the learner's life, which changes at every
 *                     average -- re-read it after each one.
 *   relocate          a round without an average: the parameters leave the published slot by one
 *                     copy into the next publish's slot (no-op when they are there).
 * Contract: the parameters ARE the served snapshot between a publish and the next average or
 * relocate, so they must not be written in that window.  The reference's own loop DOES write
 * there (README.md:18-29, examples/pytorch-cifar/main.py:130-145: update_send, the training
 * step, update_wait) and must use the write-through or full form; a resident learner needs the
 * reordered loop update_send, update_wait, step (the same gossip with each step applied after
 * the round's average instead of before it).  The Python layer records the parameters' version
 * counters at update_send and raises at update_wait when any moved (DpwaConnection,
 * DpwaPyTorchAdapter).  A publish is given the resident pointer; the split factor/lerp form is
 * refused. */
int dpwa_learner_set_resident(dpwa_learner *l, const void *init, dpwa_stream_t stream);
int dpwa_learner_resident_params(dpwa_learner *l, void **params, int *slot);
int dpwa_learner_relocate(dpwa_learner *l, dpwa_stream_t stream);

/* Split form of dpwa_learner_average for the DpwaConnection / adapter seam:
 * factor only (update_wait's return value), then lerp with the learner's coefficients. */
int dpwa_learner_factor(dpwa_learner *l, double loss, const double *loss_dev, dpwa_stream_t stream);
int dpwa_learner_lerp(dpwa_learner *l, void *flat, dpwa_stream_t stream);

/* Wire bridge.  read_snapshot: synchronous copy of the latest published
 * snapshot to host memory (header 256 B + up to payload_bytes), from any host thread --
 * RxThread's reply (conn.py:108-110); *version_out = 0 when nothing was published.
 * fetch_host: stage a snapshot received in host memory (a reference node's reply,
 * conn.py:298) as the fetch to average with; payload_bytes must equal n*sizeof(dtype).  The
 * copy waits only for the last reader of the staging buffer (not for `stream`'s queued work);
 * the host buffer may be reused on return (a page-locked one is DMA'd, and waited for). */
int dpwa_learner_read_snapshot(dpwa_learner *l, void *header_out, void *payload_out, int64_t payload_bytes,
                               uint64_t *version_out);
int dpwa_learner_fetch_host(dpwa_learner *l, const void *header, const void *payload, int64_t payload_bytes,
                            dpwa_stream_t stream);

/* Relay transport: a lock-step round's pulls spread over every xGMI link.  Each snapshot is
 * cut into `world` stripes; phase 1 (after the caller's collective that shares every rank's
 * pick, so that all publishes of the round are complete) pulls stripe `rank` of every
 * snapshot some rank needs into this rank's relay buffer; phase 2 (after a second
 * barrier) gathers this rank's peer's stripes from all ranks into staging and makes it the
 * fetch in flight (my_pick = rank averaged with, -1 none).  Both phases run on the learner's
 * side stream; picks_dev holds `world` int32 on this learner's device.
 * relay_wait makes `stream` wait for the previous round's relay work (call before the next
 * round's collective, so a slot or relay buffer is rewritten only after every reader).
 * phase2 with fuse != 0 gathers nothing yet: the next dpwa_learner_average(_through) reads the
 * peer's stripes where phase 1 left them (one kernel instead of the gather + the average; the
 * average's stream then carries the round's last reads of other ranks' relay buffers); any
 * other use of the fetch (the split factor/lerp, copy_fetched, wait_fetch) gathers first. */
int dpwa_learner_relay_enable(dpwa_learner *l, int world, int rank);
int dpwa_learner_relay_handle(dpwa_learner *l, void *handle_out, int64_t handle_len);
int dpwa_learner_relay_attach(dpwa_learner *l, int rank, int peer_id, const void *relay_handle,
                              int64_t handle_len);
int dpwa_learner_relay_attach_fds(dpwa_learner *l, int rank, int peer_id, const void *relay_handle,
                                  int64_t handle_len, const int *fds, int n_fds, int64_t chunk_bytes);
int dpwa_learner_relay_wait(dpwa_learner *l, dpwa_stream_t stream);
int dpwa_learner_relay_phase1(dpwa_learner *l, const int32_t *picks_dev, uint64_t version, int blocks,
                              dpwa_stream_t stream);
int dpwa_learner_relay_phase2(dpwa_learner *l, const int32_t *picks_dev, int my_pick, uint64_t version,
                              int blocks, int fuse);
/* Kernel timing for measurement.  time_averages allocates `capacity` begin/end event pairs
 * (0 frees them; synchronises the device).  After arm_timing, the next averaging launch
 * (average / average_through, 16-B aligned parameters) goes through hipExtLaunchKernelGGL
 * with the next free pair, so it is timed as a profiler times it, without the dispatch gaps
 * of an event pair recorded around the launch; the next publish disarms it (a round without an
 * average times nothing).  A batched dispatch (average_many) is timed with the pair of its first
 * armed learner, in call order.  read_average_times waits for and returns the recorded
 * durations (µs, launch order) and frees the pairs for reuse. */
int dpwa_learner_time_averages(dpwa_learner *l, int capacity);
int dpwa_learner_arm_timing(dpwa_learner *l);
int dpwa_learner_read_average_times(dpwa_learner *l, float *us_out, int max, int *count);
/* Bench: time the next `capacity` copying fetches (pull start to landed, on the side
 * stream; the relay is not timed) and read them back in order, in microseconds. */
int dpwa_learner_time_fetches(dpwa_learner *l, int capacity);
int dpwa_learner_read_fetch_times(dpwa_learner *l, float *us_out, int max, int *count);
/* The learner's side stream (fetches and relay phases run on it). */
int dpwa_learner_side_stream(dpwa_learner *l, dpwa_stream_t *stream);

/* Makes `stream` wait for the pull of the fetch in flight, if it copies (TxThread.fetch_wait,
 * conn.py:326-329); average/factor do this themselves -- this only lets a caller order the
 * wait before its own timing event. */
int dpwa_learner_wait_fetch(dpwa_learner *l, dpwa_stream_t stream);

/* How a copying fetch (any non-zero-copy fetch) moves its bytes: DPWA_PULL_COPY_ENGINE
 * (hipMemcpyAsync on the side stream, the default) or DPWA_PULL_KERNEL (a copy kernel of at
 * most max_blocks workgroups reading the IPC-mapped peer slot over xGMI). */
/* What a device loss pointer (`loss_dev` of publish / factor / average) points at: a float64
 * (DPWA_F64, the default) or a float32 (DPWA_F32: e.g. a training loss tensor passed as is,
 * widened exactly on the device as Python's float() widens it). */
int dpwa_learner_set_loss_dtype(dpwa_learner *l, int32_t dtype);

#define DPWA_PULL_COPY_ENGINE 0
#define DPWA_PULL_KERNEL 1
int dpwa_learner_set_pull(dpwa_learner *l, int mode, int max_blocks);

/* Reference-style seam (dpwa.py:156 returns (payload, factor) and pytorch.py:68 does the
 * arithmetic itself): copy_factor enqueues a copy of the last factor (float64) to dst_dev on
 * `stream`; copy_fetched enqueues, after the pull has landed, a copy of the payload of the fetch
 * in flight (between update_wait and the lerp) to dst_dev (n elements). */
int dpwa_learner_copy_factor(dpwa_learner *l, double *dst_dev, dpwa_stream_t stream);
int dpwa_learner_copy_fetched(dpwa_learner *l, void *dst_dev, dpwa_stream_t stream);

/* Abandons a fetch whose factor was computed but whose lerp will never be issued (the
 * caller of update_wait chose not to average); the snapshot it read may then be reused. */
int dpwa_learner_cancel(dpwa_learner *l);

/* Device pointers of the learner's blocks.  The clock is double-buffered: *clock_dev is the
 * live one and stays valid until the next factor/average.  status_word: the pinned host
 * word behind dpwa_learner_poll_status (host address), for callers that poll it directly. */
int dpwa_learner_status_word(dpwa_learner *l, int32_t **status_word);
int dpwa_learner_pointers(dpwa_learner *l, double **clock_dev, dpwa_coef **coef_dev,
                          dpwa_header **staging_header_dev, void **staging_payload_dev);
/* Synchronous reads for inspection (these DO synchronise with the learner's device). */
int dpwa_learner_read_clock(dpwa_learner *l, double *clock);
int dpwa_learner_write_clock(dpwa_learner *l, double clock);
int dpwa_learner_read_coef(dpwa_learner *l, dpwa_coef *coef);
/* Non-blocking status check: *done = 1 when the last factor computation has completed;
 * *status = the first non-OK DPWA_STATUS_* any factor computation reported since the last
 * poll (a sticky pinned host word, cleared by this call), else DPWA_STATUS_OK. */
int dpwa_learner_poll_status(dpwa_learner *l, int *done, int32_t *status);

/* ------------------------------------------------------------------------------------
 * Host scheduler: TxThread's peer choice and flow control (conn.py:178-317) plus the
 * Bernoulli fetch gate (dpwa.py:101-102), over a CPython-exact MT19937 so that a learner
 * seeded like `random.seed(seed)` draws the reference's exact sequence.
 * ------------------------------------------------------------------------------------ */
typedef struct dpwa_sched dpwa_sched;

/* outcomes reported back for a picked peer (conn.py:245-313) */
#define DPWA_CONNECT_OK 0        /* lazy connect succeeded                       conn.py:247-251 */
#define DPWA_CONNECT_REFUSED 1   /* ConnectionRefusedError: score -= 100, round ends  conn.py:253-256 */
#define DPWA_CONNECT_ERROR 2     /* other error: peer removed, round ends        conn.py:257-260 */
#define DPWA_REPLY_PAYLOAD 3     /* reply with data: score += 10, round ends      conn.py:301-302 */
#define DPWA_REPLY_EMPTY 4       /* peer had no state: score += 10, pick again    conn.py:301-302 */
#define DPWA_REPLY_TIMEOUT 5     /* socket.timeout: score -= 100, reconnect, again conn.py:304-309 */
#define DPWA_REPLY_ERROR 6       /* other error: peer removed, pick again         conn.py:311-313 */

/* static peer status for dpwa_sched_fetch (what the transport knows about each peer) */
#define DPWA_PEER_READY 0        /* up and has published                          */
#define DPWA_PEER_NO_STATE 1     /* up, nothing published yet -> empty reply       */
#define DPWA_PEER_DOWN 2         /* not up: refused when not connected, error if it was */
#define DPWA_PEER_SLOW 3         /* times out                                     */
#define DPWA_PEER_DEAD 4         /* unrecoverable: removed                        */

/* seed_key: 32-bit little-endian words of abs(seed) as CPython's random.seed(int) splits
 * it (key_len 0 means seed 0); key_len < 0 seeds from OS entropy (random.seed(None)). */
int dpwa_sched_create(dpwa_sched **out, int n_peers, const uint32_t *seed_key, int key_len,
                      double fetch_probability);
int dpwa_sched_destroy(dpwa_sched *s);
/* dpwa.py:101-102 / 118: *fetching = random() < fetch_probability */
int dpwa_sched_bernoulli(dpwa_sched *s, int *fetching);
/* conn.py:224-240: score each live peer + randint(10,1000) in insertion order, argmax,
 * tie-break randint(0, k-1).  *peer = -1 when no peers remain. *connected tells whether
 * the caller must report a CONNECT_* outcome before the REPLY_* one. */
int dpwa_sched_pick(dpwa_sched *s, int *peer, int *connected);
/* Applies an outcome for the picked peer; *round_done / *got_data say how the fetch loop
 * (conn.py:286-313) continues. */
int dpwa_sched_report(dpwa_sched *s, int peer, int outcome, int *round_done, int *got_data);
/* The whole fetch loop for one queue item (conn.py:277-315) against a static per-peer
 * status array; stops after max_attempts picks (the reference would spin forever when
 * every peer times out).  *peer_out = the peer that delivered data, or -1. */
int dpwa_sched_fetch(dpwa_sched *s, const int32_t *peer_status, int max_attempts, int *peer_out,
                     int *attempts_out);
/* flow_control_score of a peer (conn.py:190); -1 once removed */
int dpwa_sched_score(const dpwa_sched *s, int peer, int *score);
/* DpwaConnection.remove_peer (dpwa.py:98-99 -> conn.py:215-222): drop a peer for good. */
int dpwa_sched_remove(dpwa_sched *s, int peer);
/* DpwaConnection.add_peer (dpwa.py:95-96 -> conn.py:208-213): a fresh record for the peer
 * (score 1000, not connected); a removed peer is inserted again at the end of the pick order. */
int dpwa_sched_add(dpwa_sched *s, int peer);
int dpwa_sched_n_live(const dpwa_sched *s, int *n_live);
/* raw CPython-equivalent draws, for tests: random.random(), random.randint(a, b) */
/* Gossip-state checkpoint (SURVEY §5 checkpoint/resume; the reference keeps none across a
 * restart, dpwa.py:59): the scheduler's generator (CPython getstate() order), every peer's
 * flow-control score and connected/live flags, and TxThread's peer order, as 32-bit words.
 * get_state with words == NULL returns the size in *n_words; set_state validates the whole state
 * (format, peer count, score bounds, order) before changing anything.  ABI version 9. */
int dpwa_sched_get_state(const dpwa_sched *s, uint32_t *words, int max_words, int *n_words);
int dpwa_sched_set_state(dpwa_sched *s, const uint32_t *words, int n_words);
int dpwa_sched_random(dpwa_sched *s, double *out);
int dpwa_sched_randint(dpwa_sched *s, int64_t a, int64_t b, int64_t *out);

/* ------------------------------------------------------------------------------------
 * Node: DpwaConnection's per-round logic (dpwa/dpwa.py:54-156) in native code -- the
 * scheduler, the learner (bound at the first publish) and a peer table.  One call per
 * half-round keeps the host cost of a gossip round to a few microseconds.
 * ------------------------------------------------------------------------------------ */
typedef struct dpwa_node dpwa_node;

#define DPWA_NODE_PEER_UNSET 0    /* not reachable: a fetch is refused (conn.py:253-256)      */
#define DPWA_NODE_PEER_LOCAL 1    /* another node of this process (any device)                */
#define DPWA_NODE_PEER_REMOTE 2   /* IPC-attached learner of another process, lock-step rounds */

/* flags of the node calls */
#define DPWA_FLAG_EAGER 1            /* update_send/gate: start a granted fetch now (DistGroup)    */
#define DPWA_FLAG_ZERO_COPY 2        /* read a same-device local peer's slot in place              */
#define DPWA_FLAG_REUSE_SNAPSHOT 4   /* publish: flat unchanged since a write-through average      */
#define DPWA_FLAG_WRITE_THROUGH 8    /* update_wait_average: also write the next snapshot          */
#define DPWA_FLAG_PICK_ONLY 16       /* gate (EAGER): pick the peer, the caller moves the bytes    */

/* DpwaConnection.__init__ (dpwa.py:54-93) minus the model: scheduler seeded as
 * dpwa_sched_create, the interpolation config for the learner bound later. */
int dpwa_node_create(dpwa_node **out, int n_peers, const uint32_t *seed_key, int key_len,
                     double fetch_probability, const dpwa_interp *cfg);
int dpwa_node_destroy(dpwa_node *n);
/* Creates the node's learner for an n-element flat buffer of `dtype` on `device`. */
int dpwa_node_bind(dpwa_node *n, int device, int64_t numel, int32_t dtype);
/* Borrowed handles of the node's learner (NULL before bind) and scheduler. */
int dpwa_node_handles(dpwa_node *n, dpwa_learner **learner, dpwa_sched **sched);
/* How peer `peer` (scheduler index) is reached: DPWA_NODE_PEER_*; `local` for LOCAL (may be n
 * itself: a node entry at this node's own host:port, whose RxThread the reference dials like any
 * peer's -- the self-peer of configs[1]). */
int dpwa_node_set_peer(dpwa_node *n, int peer, int kind, dpwa_node *local);
/* Fault injection: force a DPWA_PEER_* status for a peer, -1 clears. */
int dpwa_node_set_fault(dpwa_node *n, int peer, int status);
/* Free-running rounds (extension of DPWA_NODE_PEER_REMOTE): the node's REMOTE peers are
 * read through `board` (see below) instead of lock-step.  peer_ranks[k] = board rank of
 * scheduler peer k; publish_timeout_ms bounds a publish's wait for readers (-1 forever).
 * board NULL returns the node to lock-step.  The node does not own the board. */
typedef struct dpwa_board dpwa_board;
int dpwa_node_set_board(dpwa_node *n, dpwa_board *board, const int32_t *peer_ranks, int publish_timeout_ms);
/* The YAML's timeout_ms (DpwaConfiguration.get_timeoutms, dpwa.py:90 -> conn.py:249) on the
 * device path (< 0 disables).  A copying pull from a local peer or through the gossip board is
 * judged when update_wait polls it (never a host wait in the normal path): landed, or out less
 * than timeout_ms (dpwa_learner_fetch_state) -> the reply with data (score +10, conn.py:301-302;
 * a pull still in flight is then waited for on the device); still in flight after timeout_ms -> a
 * socket timeout (score -100, reconnect, conn.py:304-309) and the loop picks again, the
 * re-selected pull going to a rescue lane (DPWA_FETCH_RESCUE) and being polled on the host up to
 * timeout_ms like the reference's blocking receive; a rescue pull that times out too is followed
 * by the next pick on another lane, until data, no peer or every peer removed, as TxThread
 * (conn.py:286-313).  With every lane (up to 8) still pulling, the next request waits for one to
 * land before it goes out; only a learner whose own transport stays stuck for
 * $DPWA_RESCUE_WAIT_MS (default 60000) gives that request up as a timeout and ends the round
 * without data.  Lock-step (DistGroup) pulls wait for the round's barrier, i.e. for the slowest
 * learner, not for the peer, and are not judged. */
int dpwa_node_set_timeout(dpwa_node *n, int timeout_ms);

/* update_send (dpwa.py:104-123): publish, then the Bernoulli gate; with DPWA_FLAG_EAGER a
 * granted fetch starts now (peer choice + pull on the side stream), else at update_wait.
 * Split form: publish, then (after a caller-side barrier) gate. */
int dpwa_node_update_send(dpwa_node *n, const void *flat, double loss, const double *loss_dev, int flags,
                          dpwa_stream_t stream, int *fetching);
int dpwa_node_publish(dpwa_node *n, const void *flat, double loss, const double *loss_dev, int flags,
                      dpwa_stream_t stream);
int dpwa_node_gate(dpwa_node *n, int flags, dpwa_stream_t stream, int *fetching);
/* Starts the fetch a non-eager gate granted (TxThread.run, conn.py:277-315), now instead of at
 * update_wait: a group of co-resident learners calls it once every learner of the round has
 * published, so the pull overlaps the training step (no-op when nothing is pending). */
int dpwa_node_start_fetch(dpwa_node *n, int flags, dpwa_stream_t stream);
/* update_wait (dpwa.py:125-156): *peer = the peer averaged with, or -1 for (None, 0).
 * _average fuses the adapter's lerp (pytorch.py:66-68) into the same kernel; the split
 * form computes the factor only and dpwa_node_lerp applies it. */
int dpwa_node_update_wait(dpwa_node *n, double loss, const double *loss_dev, int flags,
                          dpwa_stream_t stream, int *peer);
int dpwa_node_lerp(dpwa_node *n, void *flat, dpwa_stream_t stream);
int dpwa_node_update_wait_average(dpwa_node *n, void *flat, double loss, const double *loss_dev,
                                  int flags, dpwa_stream_t stream, int *peer);
/* update_wait_average of `count` nodes of this process whose learners share a device, in node
 * order (each node's fetch is resolved in turn, as `count` calls would), with their averages
 * enqueued as one batched dispatch (dpwa_learner_average_many).  peers[i] as *peer above. */
int dpwa_node_update_wait_average_many(dpwa_node *const *nodes, void *const *flats, const double *loss,
                                       const double *const *loss_dev, int count, int flags,
                                       dpwa_stream_t stream, int *peers);
/* Resident parameters for the node's learner (dpwa_learner_set_resident; bound, before the first
 * publish).  A resident node's update_wait_average always averages in the resident form (flat =
 * dpwa_learner_resident_params before the call) and relocates the parameters in a round without
 * an average; its split update_wait is refused. */
int dpwa_node_set_resident(dpwa_node *n, const void *init, dpwa_stream_t stream);
/* State of the current/last round: fetching flag, fetched peer (-1: none), its publish
 * number, and the picks the last fetch took. */
int dpwa_node_info(const dpwa_node *n, int *fetching, int *fetch_peer, uint64_t *fetch_version,
                   int *last_attempts);

/* ------------------------------------------------------------------------------------
 * Gossip board: free-running rounds across the processes of one node (extension).
 * Replaces the reference's always-on RxThread server (conn.py:51-172) and its publish Lock
 * (conn.py:76-79, 109-110) with a POSIX shared-memory block: the newest complete publish
 * of every rank (written by its stream after the publish), per (publisher, reader) the
 * version being pulled, and liveness (a closed entry or a dead pid is a refused
 * connection, conn.py:253-256).  No collective runs per round.
 * ------------------------------------------------------------------------------------ */
/* name: "/..." (shm_open); create != 0 on exactly one rank, before the others open. */
int dpwa_board_open(dpwa_board **out, const char *name, int world, int rank, int create);
int dpwa_board_unlink(const char *name);
/* marks this rank closed (peers see a refused connection) and unmaps */
int dpwa_board_close(dpwa_board *b);
/* hipHostRegister the block for stream writes from `device` (needed before a device
 * advertise/release) */
int dpwa_board_register(dpwa_board *b, int device);
/* DPWA_PEER_DOWN / NO_STATE / READY for rank r */
int dpwa_board_status(dpwa_board *b, int r, int32_t *status);
/* raw view of rank r: its newest complete publish, our read mark on it, liveness */
int dpwa_board_read(dpwa_board *b, int r, uint64_t *version, uint64_t *reading_by_me, int32_t *alive);
/* reader: a version of r that r will not overwrite until released (0 = never published) */
int dpwa_board_acquire(dpwa_board *b, int r, uint64_t *version);
/* reader: clear the read mark on r after the work on `stream` (host != 0: now) */
int dpwa_board_release(dpwa_board *b, int r, dpwa_stream_t stream, int host);
/* publisher: wait until publish `next` may rewrite its slot (timeout_ms < 0: forever) */
int dpwa_board_publish_wait(dpwa_board *b, uint64_t next, int timeout_ms);
/* publisher: announce publish `version` after the work on `stream` (host != 0: now) */
int dpwa_board_advertise(dpwa_board *b, uint64_t version, dpwa_stream_t stream, int host);

#ifdef __cplusplus
}
#endif

#endif /* DPWA_HIP_H */
