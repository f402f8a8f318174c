// xyws_stream.h — run-parallel stream decoder (xyws_stream.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "xyws.h"

// Scratch owned by a context: one record + one flag per run, a ticket and a
// device error word.
struct stream_scratch {
  void* mem;            // device allocation
  uint64_t bytes;
  uint64_t max_runs;    // runs the allocation covers
  int ncu;              // compute units of the context's device (runs per launch)
  void* fmem;           // frame-start lists for descriptor emission (grown with the caller's cap)
  uint64_t fbytes;
  // decoder choice: pinned host words the finisher of every call writes
  // ({epoch, batch bytes, smallest, largest last-frame size, decoder}) and
  // their device address; null when the pinned allocation failed (then the
  // run decoder serves every call)
  volatile uint64_t* pol_h;
  uint64_t* pol_d;
  void* lmem;           // lattice decoder: scratch words + one result word per segment
  uint64_t lmax_segs;
};

void stream_scratch_init(stream_scratch* s, int device);
void stream_scratch_free(stream_scratch* s);
int stream_scratch_reserve(stream_scratch* s, uint64_t max_batch_bytes);
int stream_scratch_reserve_frames(stream_scratch* s, uint64_t max_batch_bytes, uint64_t max_frames);
// sticky device error word of this scratch (bit 1: an inter-workgroup wait
// timed out, bit 2: a run record was not written by its call); clear: reset
// it after reading (the device must be idle)
uint32_t stream_scratch_error(stream_scratch* s, bool clear);
#define XYWS_NSTATS 48
int stream_scratch_stats(stream_scratch* s, uint64_t out[XYWS_NSTATS]);
int64_t stream_scratch_records(stream_scratch* s, uint64_t* out, uint64_t max_runs);
// {the device policy word (HW_DPOL), lattice calls handed whole to the run
// decoder on it, ... by the prologue's checks, lattice calls whose segment
// loops ran in 75 KiB segments, ... in 120 KiB segments}; synchronizes the
// device
int stream_scratch_lattice(stream_scratch* s, uint64_t out[5]);
// xyws_unmask's claim counter pair (u32 claims, u32 workgroups done; zeroed at
// allocation, reset by the kernel's last workgroup) in this scratch
int stream_scratch_unmask_counter(stream_scratch* s, bool capturing, uint32_t** out);

// Internal decode options (not part of include/xyws.h):
#define XYWS_OPT_STATS 0x100u      // count speculation/repair events (xyws_debug_stats)
#define XYWS_OPT_SMALL_SEG 0x200u  // 1 KiB segments, one per run: exercises run-boundary
                                   // speculation and repair on small test inputs
#define XYWS_OPT_NO_DENSE0 0x1000u  // experiment (run decoder): the stride pass first in every run's first
                                   // segment even after a call of small mixed-size frames (no dense0 hint)
#define XYWS_OPT_NO_LATENTRY 0x4000u // experiment (run decoder): no lattice entry (find_entry scans every run)
#define XYWS_OPT_WG1024 0x8000u    // the run decoder in its default geometry (one 1024-thread workgroup per CU),
                                   // whatever the geometry choice (wg512_preferred) would take
#define XYWS_OPT_RUNS_NOWAIT 0x10000u // experiment (run decoder): a serial-chase segment's stores do not wait for the
                                   // next segment's loads (the dense pass's behaviour)
#define XYWS_OPT_NO_STORE 0x20000u // diagnostics: decode without writing (timing split only)
#define XYWS_OPT_WG512 0x40000u    // two 512-thread workgroups per CU, 64 KiB segments
#define XYWS_OPT_DIAG 0x80000u     // diagnostics: no prefetch during the prologue scan (timing only)
#define XYWS_OPT_TEST_GIVEUP 0x100000u // tests: odd runs give up on their successor at once (the path
                                       // of a successor whose workgroup has not started; finish bridges it)
#define XYWS_OPT_NO_LATTICE 0x200000u   // experiment (run decoder): no lattice passes (row table and walk only)
#define XYWS_OPT_STEAL 0x400000u       // work stealing between runs (off by default: measured no faster on c1-c4)
#define XYWS_OPT_TEST_STEAL 0x800000u  // tests: stealing on, every fourth run starts late, pieces of 1 segment and up
#define XYWS_OPT_LAT_NOGATE 0x1000000u  // (set by the lattice kernel only, from the device policy word) no
                                        // first-segment gate: the previous call on the stream was the lattice's
#define XYWS_OPT_LAT_GATE 0x2000000u    // experiment (lattice decoder): the first-segment gate whatever the
                                        // previous call found
#define XYWS_OPT_LATX_NOCHK 0x8000000u  // experiment (lattice decoder): no check of lattice points 1 and 2 up front
#define XYWS_OPT_IOV_PIECES 0x10000000u  // xyws_decode_stream_iov: the pieces in place one by one (no descriptors)
#define XYWS_OPT_IOV_STAGE 0x20000000u   // xyws_decode_stream_iov: gather, decode, scatter whatever the pieces
#define XYWS_OPT_BIGSCAN 0x4000000u  // tests (entry scans): one filter pass per segment, whatever the previous
                                     // call found
#define XYWS_OPT_NO_BIGSCAN 0x40000000u // experiment (entry scans): the window-0 pass whatever the previous call found
#define XYWS_OPT_RUNS 0x80000000u     // the run decoder, whatever the decoder choice would take
#define XYWS_OPT_LATTICE 0x400u      // the lattice decoder first, whatever the decoder choice would take
#define XYWS_OPT_NO_LATDEC 0x800u    // never the lattice decoder
#define XYWS_OPT_TEST_LATSPEC 0x10u  // tests (lattice decoder): every store speculative (no first-segment gate, no
                                     // failing-point filter): a broken lattice is undone by the end-of-work check
#define XYWS_OPT_WG256 0x8u  // the run decoder in four 256-thread workgroups per CU on 16 KiB segments
#define XYWS_OPT_LATX_ONLY 0x80u  // timing experiment only (wrong bytes after a redirect): no run decoder after the lattice
#define XYWS_OPT_TEST_LATDUMP 0x20u  // tests (lattice decoder): a workgroup never undoes its own speculative
                                    // stores at its end: every list goes to the finisher
#define XYWS_OPT_LATX_NOWORK 0x40u  // timing experiment only (wrong bytes): the lattice decoder's data waves skip
                                    // the checks and the XOR (its data path and control alone)
#define XYWS_OPT_REDIRECT 0x2000u    // (set by stream_decode_fused only) the run decoder after the lattice decoder:
                                     // it reads the lattice's redirect record first
int stream_decode_fused(stream_scratch* s, uint8_t* base, uint64_t lo, uint64_t hi,
                        const xyws_carry* cin, xyws_carry* cout, xyws_frame* frames, uint64_t cap,
                        uint64_t* nframes, uint32_t opts, hipStream_t stream);
