// A per-device side stream and its events, for the native trainers' overlap of
// one local step's optimizer update (HBM-bound) with the next step's forward
// (MFMA / latency-bound): the update runs on the side stream parameter group
// by parameter group, each group's event recorded after it, and the forward
// waits on a group's event before its first use of those parameters.  Every
// side-stream branch is joined back into the caller's stream within the same
// call, so the entry points stay stream-ordered and capturable in a HIP graph
// (fork / join through events is how a capture spans two streams).
//
// The stream and events are created once per device, outside any capture
// (flr_*_workspace queries create them; a call that finds none while its
// stream is capturing runs the update on the caller's stream instead — same
// results, no overlap).
//
// One stream and one event set per device, shared by every trainer of the
// process: with FLR_SGD_OVERLAP=1 at most one training call may be in flight
// per device at a time (two concurrent callers would record and wait on the
// same events).  A model with more parameter groups than NEV - 1 updates on
// the caller's stream (no overlap, same results).
//
// Off by default (FLR_SGD_OVERLAP=1 turns it on).  Measured at C3 on MI355X
// (tools/gpu_r3_k.sh, gpu_r3_l.sh): 79 % of the optimizer's kernel time does
// run concurrently with the forward's kernels, but both slow down by as much
// (summed kernel time 59.3 -> 69.1 ms per round) and the round time is
// unchanged (61.6 vs 61.8-62.2 ms); a side stream created with a priority
// (either end of the range) made the round 50 % slower.
#pragma once

#include <cstdlib>
#include <mutex>

#include "flr_common.h"

namespace flr {

struct SideStream {
  static constexpr int NEV = 48;
  hipStream_t s = nullptr;
  hipEvent_t ev[NEV] = {};
};

// The optimizer update on a side stream under the next step's forward
// (FLR_SGD_OVERLAP=1) measured no faster: tools build only.
inline bool side_overlap_enabled() {
#ifdef FLR_ABLATION
  const char* e = flr::knob("FLR_SGD_OVERLAP");
  return e && e[0] == '1';
#else
  return false;
#endif
}

// The current device's side stream; created on first use when create is set
// (never during a capture of `st`).  nullptr: none (or overlap disabled).
inline SideStream* side_stream(bool create, hipStream_t st = nullptr) {
  if (!side_overlap_enabled()) return nullptr;
  static SideStream pool[64];
  static bool made[64] = {};
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (made[dev]) return &pool[dev];
  if (!create) return nullptr;
  if (st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  }
  SideStream& ss = pool[dev];
  if (hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  for (int i = 0; i < SideStream::NEV; ++i)
    if (hipEventCreateWithFlags(&ss.ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
  made[dev] = true;
  return &ss;
}

// The text-branch stream of the ResNet + GRU trainer (train_clients.hip): the
// embedding + GRU forward and backward run on it beside the image trunk (the
// recurrence is a chain of small latency-bound launches that leaves most of the
// chip idle), forked from and joined to the caller's stream by events (graph-
// capturable).  One per device, created outside any capture; one training
// call per device at a time.  FLR_TEXT_STREAM=0: everything on the caller's
// stream (A/B, read per call).
struct TextStream {
  // forward fork / join, backward fork / join; 4 .. NEV - 2: the trunk's last
  // weight gradients forked onto it (idle by then), NEV - 1 their join
  static constexpr int NEV = 8;
  hipStream_t s = nullptr;
  hipEvent_t ev[NEV] = {};
};

inline bool text_stream_enabled() {
  const char* e = flr::knob("FLR_TEXT_STREAM");
  return !(e && e[0] == '0');
}

inline TextStream* text_stream(bool create, hipStream_t st = nullptr) {
  if (!text_stream_enabled()) return nullptr;
  static TextStream pool[64];
  static bool made[64] = {};
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (made[dev]) return &pool[dev];
  if (!create) return nullptr;
  if (st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  }
  TextStream& ts = pool[dev];
  if (hipStreamCreateWithFlags(&ts.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  for (int i = 0; i < TextStream::NEV; ++i)
    if (hipEventCreateWithFlags(&ts.ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
  made[dev] = true;
  return &ts;
}

// The weight-gradient stream of the native trainers: every tap-major conv's
// weight gradient (ResNet + GRU) and every ViT layer's weight / bias gradients
// (ViT + BERT) run on it, forked after the layer's output gradient is ready,
// while the caller's stream continues down the data-gradient chain (the
// backward's critical path); joined before the clip + SGD step.  Per device,
// created outside any capture; FLR_WGRAD_STREAM=0: off (A/B).
struct WgradStream {
  static constexpr int NEV = 128;
  hipStream_t s = nullptr;
  hipEvent_t ev[NEV] = {};
};

inline bool wgrad_stream_enabled() {
  const char* e = flr::knob("FLR_WGRAD_STREAM");
  return !(e && e[0] == '0');
}

inline WgradStream* wgrad_stream(bool create, hipStream_t st = nullptr) {
  if (!wgrad_stream_enabled()) return nullptr;
  static WgradStream pool[64];
  static bool made[64] = {};
  static std::mutex mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (made[dev]) return &pool[dev];
  if (!create) return nullptr;
  if (st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  }
  WgradStream& ws = pool[dev];
  if (hipStreamCreateWithFlags(&ws.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  for (int i = 0; i < WgradStream::NEV; ++i)
    if (hipEventCreateWithFlags(&ws.ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
  made[dev] = true;
  return &ws;
}

}  // namespace flr
