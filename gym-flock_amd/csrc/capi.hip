// C-ABI of libgymflock.so (include/gymflock.h): handle lifecycle, device buffers,
// stream-ordered launches, host transfers, RCCL metrics path and error reporting.
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "device_alloc.h"
#include "flock_internal.h"
#include "gymflock.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int fail_hip(const char* what, hipError_t e) {
  return fail(GF_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define GF_HIP(expr)                                        \
  do {                                                      \
    hipError_t e_ = (expr);                                 \
    if (e_ != hipSuccess) return fail_hip(#expr, e_);       \
  } while (0)

// Reward ring: the t-th reward-writing launch writes slot t % kRewardSlots. The metrics
// all-gather ships every step written since the previous gather (at most kRewardSlots).
constexpr int kRewardSlots = 64;
// fe_comm_init's bound on the communicator's creation, its shard-size exchange and every
// later wait for a collective
constexpr double kCommInitTimeoutS = 300.0;

}  // namespace

namespace gf {
// Shared with the Coverage C-ABI (cov_capi.hip): one thread-local error message.
int set_error(int code, const std::string& msg) { return fail(code, msg); }
}  // namespace gf

struct fe_handle {
  fe_config cfg{};
  hipStream_t stream = nullptr;
  hipStream_t comm_stream = nullptr;
  // Split steps: the step's env batch goes out as two launches, envs [0, B0) on
  // `stream` and [B0, B) on `stream2`, so one launch's ramp and tail overlap the other's
  // body (175.8 vs 196.0 us per config-2 step). The halves only depend on
  // their own previous step; `stream` waits for `stream2` (join) before any other work.
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_s2 = nullptr;           // stream2 -> stream join
  hipEvent_t ev_main = nullptr;         // stream -> stream2 ordering
  int nsplit = 2;                       // launches per step (fe_set_streams)
  bool s2_pending = false;              // stream2 holds work `stream` has not waited for
  bool main_dirty = true;               // `stream` holds work stream2 has not waited for
  bool dephase = true;                  // the next split step starts the halves apart (other
                                        // work or a single launch came before it)
  bool other_work = true;               // non-step work was enqueued since the last step:
                                        // the next step goes out as one launch (a split
                                        // step would only wait on it across streams)
  hipEvent_t tw[2] = {nullptr, nullptr};  // split-step timing window (fe_kernel_timing)
  int64_t tw_steps = 0;
  double* x[2] = {nullptr, nullptr};
  int cur = 0;
  void* u = nullptr;                    // (B,N,2) up to float64
  double* ctrl[2] = {nullptr, nullptr};
  int ccur = 0;
  float* sv = nullptr;
  float* net = nullptr;
  double* reward_ring = nullptr;        // kRewardSlots x B
  int rslot = 0;
  int64_t steps_written = 0;            // reward-writing launches so far (slot = count % slots)
  // kNN outputs, one pair per state buffer: knn_idx[i] / knn_obs[i] belong to x[i], so
  // a fused step (which writes those of its output state) never overlaps the rim kNN of
  // the previous state, and the kread events that guard x[i] guard them too
  int32_t* knn_idx[2] = {nullptr, nullptr};
  float* knn_obs[2] = {nullptr, nullptr};
  // each ranked row's k-th nearest r2 (0: unknown), by state buffer: a fused step reads
  // the one of two states back (complete: the step waits for that state's kNN) to pick
  // the rows it ranks beyond their neighbours, and writes its own
  float* knn_r2[2] = {nullptr, nullptr};
  uint8_t* knn_rimflag[2] = {nullptr, nullptr};  // per state buffer: blocks with rim rows
  double* vel_diffs = nullptr;
  double* min_dists = nullptr;
  int32_t* degree = nullptr;
  int u_resident_f64 = -1;              // dtype of the resident actions (-1: none)
  bool has_state = false, has_ctrl = false, has_obs = false, has_knn = false;
  bool obs_on_host = false;             // the last launch wrote state_values / network to
                                        // host arrays only (fe_step_host): device copies stale
  int R = 0, T = 0, bpe = 0;
  int knn_exact = 0;                    // the fused kNN is exact in the step (gf::step_knn_exact)
  size_t BN = 0;
  int diag = 0;                         // ablation switches (diagnostic build only, fe_diag)
  int prefetch = 0;                     // tile loads one tile ahead (N >= 16 tiles)
  int store_fast[2] = {0, 1};           // fast network store loop: plain step / with controller
  // kernel timing (bench roofline)
  bool timing = false;
  int timing_stride = 1;                // sample every timing_stride-th launch
  int64_t timing_count = 0;
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  // RCCL metrics path. Shards may differ in size: every gathered block is padded to the
  // largest shard (max_envs), rank r's entries past its n_envs are zero.
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  int max_envs = 0;
  std::vector<int32_t> shard_sizes;     // every rank's n_envs (fe_comm_init's exchange)
  double comm_timeout = kCommInitTimeoutS;  // bound on every wait for a collective
  // The step streams never wait on the side stream on the device: a collective stuck on
  // a dead peer (and, through it, everything queued behind it) must not stall the steps.
  // A step about to overwrite a ring slot that a gather's staging copy has not read yet
  // waits for that copy on the host, bounded by comm_timeout (next_reward_slot); normally
  // the copy finished long before (the slot was written kRewardSlots steps ago).
  double* gsend = nullptr;              // kRewardSlots x max_envs: the gathered steps, padded
  std::string comm_lost;                // why the metrics path was torn down (a timed-out wait)
  double* gather = nullptr;             // nranks x kRewardSlots x max_envs
  hipEvent_t step_ev = nullptr;
  hipEvent_t step_ev2 = nullptr;        // the gather's wait on stream2 (split steps)
  hipEvent_t h2d_ev = nullptr;          // completion of the borrowed host-action copy
  // Host actions of split steps (fe_step without FE_U_*): copied on a stream of their own
  // into one of two device buffers, so the copy for step t+1 runs while step t computes;
  // buffer k is rewritten only after both halves of the step that read it (two calls
  // back) have finished (ev_uread), and both halves of its step wait for its copy.
  hipStream_t ustream = nullptr;
  void* ubuf[2] = {nullptr, nullptr};   // (B,N,2) up to float64 each
  hipEvent_t ev_ucopy[2] = {nullptr, nullptr};
  hipEvent_t ev_uread[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  bool uread_live[2] = {false, false};
  int ucur = 0;
  // ring slots a reward gather's staging copy still reads: steps [first, ...) until the
  // copy kernel (on the side stream) has stored `seq` into completion word kWordRing
  struct RingRead {
    int64_t first;
    uint32_t seq;
  };
  std::deque<RingRead> ring_reads;
  // The side stream's completion words (kWord*): page-locked (mapped, coherent), each
  // stored by a kernel on the side stream with a system-scope release once the work
  // before it is done, and polled by the host instead of querying events; never freed
  // once a communicator was aborted (an abandoned kernel may still store into them)
  uint32_t* stage_done = nullptr;
  uint32_t* stage_done_dev = nullptr;
  uint32_t stage_seq[4] = {0, 0, 0, 0};  // the last sequence number issued per word
  int64_t gathered_upto = 0;            // steps before this one were shipped (or skipped)
  bool ag_issued = false;
  int last_count = 0;
  double* stats_sum = nullptr;          // (B,2) get_stats means per env (fe_stats_summary)
  double* ssend = nullptr;              // (max_envs,2) the stats gather's padded send block
  double* stats_gather = nullptr;       // nranks x max_envs x 2 (fe_allgather_stats)
  bool sg_pending = false;
  // fe_debug_comm_gate: a bounded spin kernel on comm_stream, released by this page-locked
  // flag, stands in for a collective whose peer stopped responding (tests only)
  unsigned* gate_flag = nullptr;
  // fe_debug_comm_state: what the ring-slot reuse and the gathers saw (tests only)
  int32_t dbg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // fe_step_host*: the launch's completion flag (done_flag.h), allocated on first use: the
  // device counter, the page-locked word and its mapped address
  int32_t* fin_cnt = nullptr;
  int32_t* fin_host = nullptr;
  int32_t* fin_dev = nullptr;
  int32_t fin_seq = 0;
  // flocking variant (fe_set_variant / fe_set_dt)
  bool has_variant = false;
  fe_variant var{};
  double* dt_env = nullptr;             // (B) per-env dt
  bool dt_per_env = false;
  // packed output mode (FE_PACKED_NETWORK) and the kNN step's adjacency: two buffers,
  // so a step can write one while the kNN of the previous step reads the other
  uint64_t* adj_bits[2] = {nullptr, nullptr};  // (B,N,Wn)
  int32_t* pdeg[2] = {nullptr, nullptr};       // (B,N)
  int bits_cur = 0;                     // buffer of the latest bits / degrees
  bool has_packed = false;
  // Flocking-v0 pipelining: the kNN of step t runs on kstream, after both halves of
  // step t and beside step t+1. A step that writes the state buffer x[i] (or a bits
  // buffer) an unfinished kNN reads waits for that kNN's event first; every other API
  // call joins kstream into `stream` (use_dev).
  // The fused step's rim kNN (mode 2) is not on kstream: after a split step it goes out
  // as two launches on the step streams themselves, envs [0, B0) behind `stream`'s half
  // and [B0, B) behind stream2's, so each half of the next step follows its own rim by
  // stream order and the halves keep drifting out of phase (Flocking-v0).
  hipStream_t kstream = nullptr;
  hipEvent_t ev_kin[2] = {nullptr, nullptr};  // stream / stream2 -> kstream
  hipEvent_t ev_kjoin = nullptr;              // kstream -> stream
  bool k_pending = false;                     // kstream holds work `stream` has not waited for
  int last_b0 = 0;                            // B0 of the last launch if it was split, else 0
  struct KnnReader {
    hipEvent_t ev = nullptr;                  // the kNN launch on kstream
    bool live = false;
    unsigned bmask = 0;                       // bits buffers it reads
  } kread[2];                                 // by the state buffer x[i] the kNN reads
};

namespace {

// fe_get_outputs(FE_OUT_MAPPED): the step's outputs into page-locked host arrays through
// their mapped addresses, 16-byte stores where both sides allow (grid-stride).
struct OutCopy {
  const float* src[2];
  float* dst[2];
  size_t n[2];  // floats
  const double* rsrc;
  double* rdst;
  int nr;
};

__global__ __launch_bounds__(256) void out_copy_kernel(OutCopy c) {
  const size_t t0 = (size_t)blockIdx.x * 256 + threadIdx.x, st = (size_t)gridDim.x * 256;
  for (int a = 0; a < 2; ++a) {
    if (!c.dst[a]) continue;
    const float* s = c.src[a];
    float* d = c.dst[a];
    const size_t n = c.n[a];
    if (((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0) {
      const size_t n4 = n >> 2;
      for (size_t k = t0; k < n4; k += st) reinterpret_cast<float4*>(d)[k] = reinterpret_cast<const float4*>(s)[k];
      for (size_t k = (n4 << 2) + t0; k < n; k += st) d[k] = s[k];
    } else {
      for (size_t k = t0; k < n; k += st) d[k] = s[k];
    }
  }
  if (c.rdst)
    for (size_t k = t0; k < (size_t)c.nr; k += st) c.rdst[k] = c.rsrc[k];
}

// The device address of page-locked host memory, or nullptr (pageable: its failed
// lookup's error is cleared so later launch checks do not see it).
void* mapped_ptr(void* p) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

// `stream` waits for the second half-batch stream (enqueue only, no host sync).
int join_s2(fe_handle* h) {
  if (h->s2_pending) {
    GF_HIP(hipEventRecord(h->ev_s2, h->stream2));
    GF_HIP(hipStreamWaitEvent(h->stream, h->ev_s2, 0));
    h->s2_pending = false;
  }
  return GF_OK;
}

// `stream` waits for the kNN stream (enqueue only). Later work on `stream` (and, through
// main_dirty, on stream2) is then ordered after every kNN launched so far.
int join_k(fe_handle* h) {
  if (h->k_pending) {
    GF_HIP(hipEventRecord(h->ev_kjoin, h->kstream));
    GF_HIP(hipStreamWaitEvent(h->stream, h->ev_kjoin, 0));
    h->k_pending = false;
  }
  for (auto& r : h->kread) r.live = false, r.bmask = 0;
  return GF_OK;
}

// Whether the next step launch of B envs goes out as two half-batch launches.
bool split_next(const fe_handle* h, int B) { return h->nsplit > 1 && B >= 2 && h->stream2 && !h->other_work; }

// Before a step writes x[xw] (xw < 0: no state write) and bits buffer bw (bw < 0: none):
// both step streams wait for the unfinished kNN launch (on kstream) that reads them. The
// fused step's rim kNN runs on the step streams and needs no wait.
int wait_knn_readers(fe_handle* h, int xw, int bw) {
  for (int i = 0; i < 2; ++i) {
    auto& r = h->kread[i];
    if (r.live && (i == xw || (bw >= 0 && ((r.bmask >> bw) & 1u)))) {
      GF_HIP(hipStreamWaitEvent(h->stream, r.ev, 0));
      GF_HIP(hipStreamWaitEvent(h->stream2, r.ev, 0));
      r.live = false;
      r.bmask = 0;
    }
  }
  return GF_OK;
}

// Every API call except the step launches: the device, and `stream` ordered after all
// of the handle's outstanding work; what it enqueues is ordered before the next
// second-half launch (main_dirty).
int use_dev(fe_handle* h) {
  GF_HIP(hipSetDevice(h->cfg.device));
  if (int rc = join_s2(h)) return rc;
  if (int rc = join_k(h)) return rc;
  h->main_dirty = true;
  h->dephase = true;
  h->other_work = true;
  return GF_OK;
}

// The step path: only the device (the halves order themselves, see launch_step_split).
int use_dev_step(fe_handle* h) {
  GF_HIP(hipSetDevice(h->cfg.device));
  return GF_OK;
}

template <class T>
int dalloc(T** p, size_t count) {
  if (count == 0) {
    *p = nullptr;
    return GF_OK;
  }
  hipError_t e = gf::device_alloc(reinterpret_cast<void**>(p), count * sizeof(T));
  if (e != hipSuccess) return fail(GF_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return GF_OK;
}

// ---- the process's communicator worker
// ncclCommAbort runs on one thread per process that lives until the process exits (never
// on a short-lived thread: RCCL's own threads may keep using the HIP thread-local state of
// the thread that called into it, and a thread that exited under them corrupted the heap
// once torch's HIP runtime was bound). The worker and its queue are never
// destroyed, so the thread outlives static destruction.
struct CommWorker {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<ncclComm_t, int>> q;  // (communicator, device)
};

CommWorker* comm_worker() {
  static CommWorker* w = [] {
    auto* p = new CommWorker();
    std::thread([p] {
      for (;;) {
        std::pair<ncclComm_t, int> job;
        {
          std::unique_lock<std::mutex> l(p->mu);
          p->cv.wait(l, [p] { return !p->q.empty(); });
          job = p->q.front();
          p->q.pop_front();
        }
        hipSetDevice(job.second);
        ncclCommAbort(job.first);
      }
    }).detach();
    return p;
  }();
  return w;
}

void abort_comm_later(ncclComm_t c, int device) {
  CommWorker* w = comm_worker();
  {
    std::lock_guard<std::mutex> l(w->mu);
    w->q.emplace_back(c, device);
  }
  w->cv.notify_one();
}

// A thread that called into RCCL's initialisation parks here for the rest of the process
// instead of exiting (the same thread-local-state reason as the worker above).
[[noreturn]] void park_thread() {
  static std::mutex* m = new std::mutex();
  static std::condition_variable* cv = new std::condition_variable();
  std::unique_lock<std::mutex> l(*m);
  for (;;) cv->wait(l);
}

using Clock = std::chrono::steady_clock;

Clock::time_point deadline_in(double seconds) {
  return Clock::now() + std::chrono::microseconds(static_cast<int64_t>(seconds * 1e6));
}

// Every collective on the side stream complete, polled against the collective timeout and
// the communicator's async error; false when it expired (a peer stopped responding).
bool comm_stream_drained(fe_handle* h) {
  if (!h->comm_stream) return true;
  const auto deadline = deadline_in(h->comm_timeout);
  for (int spin = 0;; ++spin) {
    const hipError_t q = hipStreamQuery(h->comm_stream);
    if (q != hipErrorNotReady) return q == hipSuccess;
    ncclResult_t st = ncclSuccess;
    if (h->comm && (ncclCommGetAsyncError(h->comm, &st) != ncclSuccess || (st != ncclSuccess && st != ncclInProgress)))
      return false;
    if (Clock::now() > deadline) return false;
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// Tear down the metrics path: the communicator (aborted when a collective may never
// complete, else destroyed once the side stream has drained) and everything fe_comm_init
// made for it, so that a later fe_comm_init starts from scratch.
//
// abort: a collective (or the initialisation) may never finish because a peer is gone.
// The communicator is then aborted on the process's communicator worker, and the side
// stream, its events and the buffers its collectives use are abandoned rather than
// synchronised or freed (a kernel of the aborted collective may still touch them), so
// that this call cannot hang; the step streams never wait on the side stream. A
// non-abort release whose side stream does not drain within the collective timeout
// becomes an abort.
void comm_release(fe_handle* h, bool abort) {
  if (!abort && h->comm && !comm_stream_drained(h)) abort = true;
  if (abort) {
    if (h->comm) abort_comm_later(h->comm, h->cfg.device);
    h->comm = nullptr;
    h->comm_stream = nullptr;
    h->step_ev = h->step_ev2 = nullptr;
    h->ring_reads.clear();  // copies the side stream may still run: abandoned, and so
    h->stage_done = h->stage_done_dev = nullptr;  // is the word they would store into
    h->gsend = h->gather = h->ssend = h->stats_gather = nullptr;
  }
  if (h->comm) {
    ncclCommDestroy(h->comm);
    h->comm = nullptr;
  }
  if (h->comm_stream) {
    hipStreamSynchronize(h->comm_stream);  // drained above
    hipStreamDestroy(h->comm_stream);
    h->comm_stream = nullptr;
  }
  for (hipEvent_t* e : {&h->step_ev, &h->step_ev2})
    if (*e) {
      hipEventDestroy(*e);
      *e = nullptr;
    }
  h->ring_reads.clear();
  for (double** p : {&h->gsend, &h->gather, &h->ssend, &h->stats_gather})
    if (*p) {
      hipFree(*p);
      *p = nullptr;
    }
  h->ag_issued = h->sg_pending = false;
  h->last_count = 0;
  h->nranks = 1;
  h->rank = 0;
  h->max_envs = 0;
  h->shard_sizes.clear();
}

void release(fe_handle* h) {
  if (!h) return;
  hipSetDevice(h->cfg.device);
  if (h->stream) hipStreamSynchronize(h->stream);
  if (h->stream2) hipStreamSynchronize(h->stream2);
  if (h->kstream) hipStreamSynchronize(h->kstream);
  if (h->ustream) hipStreamSynchronize(h->ustream);
  comm_release(h, false);
  void* bufs[] = {h->x[0], h->x[1], h->u, h->ctrl[0], h->ctrl[1], h->sv, h->net, h->reward_ring,
                  h->knn_idx[0], h->knn_idx[1], h->knn_obs[0], h->knn_obs[1], h->knn_r2[0], h->knn_r2[1], h->knn_rimflag[0], h->knn_rimflag[1], h->vel_diffs, h->min_dists, h->degree, h->stats_sum, h->dt_env,
                  h->adj_bits[0], h->adj_bits[1], h->pdeg[0], h->pdeg[1]};
  for (void* p : bufs)
    if (p) hipFree(p);
  if (h->fin_cnt) hipFree(h->fin_cnt);
  if (h->fin_host) hipHostFree(h->fin_host);
  if (h->stage_done) hipHostFree(h->stage_done);  // (the side stream drained or was never used)
  for (hipEvent_t e : h->ev) hipEventDestroy(e);
  if (h->h2d_ev) hipEventDestroy(h->h2d_ev);
  for (hipEvent_t e : {h->ev_s2, h->ev_main, h->tw[0], h->tw[1], h->ev_kin[0], h->ev_kin[1], h->ev_kjoin,
                       h->kread[0].ev, h->kread[1].ev, h->ev_ucopy[0], h->ev_ucopy[1], h->ev_uread[0][0],
                       h->ev_uread[0][1], h->ev_uread[1][0], h->ev_uread[1][1]})
    if (e) hipEventDestroy(e);
  for (void* p : h->ubuf)
    if (p) hipFree(p);
  if (h->ustream) hipStreamDestroy(h->ustream);
  if (h->kstream) hipStreamDestroy(h->kstream);
  if (h->stream) hipStreamDestroy(h->stream);
  if (h->stream2) hipStreamDestroy(h->stream2);
  delete h;
}

int check_env(const fe_handle* h, int env) {
  if (env >= h->cfg.n_envs) return fail(GF_EINVAL, "env index out of range");
  return GF_OK;
}

double* cur_reward(fe_handle* h) { return h->reward_ring + (size_t)h->rslot * h->cfg.n_envs; }

// completion words of the side stream (fe_handle::stage_done)
enum { kWordRing = 0, kWordStatsCopy = 1, kWordRewardGather = 2, kWordStatsGather = 3 };
int stage_wait(fe_handle* h, int word, uint32_t seq, const char* what);

// Whether the side-stream work numbered `seq` on completion word `word` is done (each
// word's kernels run in order on the side stream, so the word only grows).
bool stage_complete(const fe_handle* h, int word, uint32_t seq) {
  return static_cast<int32_t>(__atomic_load_n(h->stage_done + word, __ATOMIC_ACQUIRE) - seq) >= 0;
}

int no_comm(const fe_handle* h) {
  return fail(GF_ESTATE, "no communicator (fe_comm_init not called, or it was torn down" +
                             (h->comm_lost.empty() ? std::string(")") : ": " + h->comm_lost + ")"));
}

// Advance the reward ring before a launch that writes rewards. The slot last held the
// step kRewardSlots launches back. A reward gather's staging copy (on the side stream,
// behind the previous collectives) that may still read it has normally finished long
// ago: its event is queried on the host. If not, the host waits for it, bounded by the
// collective timeout; on expiry (a collective stuck on a peer that stopped responding)
// the metrics path is torn down (the communicator aborted, the reason kept for the next
// metrics call) and the step goes on. The step streams never wait on the side stream on
// the device, so nothing queued behind a stuck collective can stall them.
int next_reward_slot(fe_handle* h) {
  const int64_t s = h->steps_written;
  h->rslot = static_cast<int>(s % kRewardSlots);
  while (!h->ring_reads.empty() && h->ring_reads.front().first <= s - kRewardSlots) {
    const uint32_t seq = h->ring_reads.front().seq;
    const bool done = stage_complete(h, kWordRing, seq);
    h->dbg[0]++;
    h->dbg[1] = done ? 1 : 0;
    h->dbg[2] = -1;
    if (!done) {
      h->dbg[2] = stage_wait(h, kWordRing, seq, "reward all-gather staging copy (ring slot reuse)");
      if (h->dbg[2] == GF_ECOMM) {
        h->comm_lost = g_err;  // comm_release emptied ring_reads: the step goes on
        break;
      }
      if (h->dbg[2] != GF_OK) return h->dbg[2];
    }
    h->ring_reads.pop_front();
  }
  h->steps_written = s + 1;
  return GF_OK;
}

// Packed-output buffers on first use: adjacency bits (FE_PACKED_NETWORK, or the kNN
// step) and their degrees. A launch writes the buffer pair the latest bits are not in;
// *bw is its index (-1: no bits written).
int packed_outputs(fe_handle* h, bool bits, gf::StepArgs& a, int* bw) {
  *bw = -1;
  if (!bits) return GF_OK;
  const int k = h->bits_cur ^ 1;
  if (!h->adj_bits[k])
    if (int rc = dalloc(&h->adj_bits[k], h->BN * ((h->cfg.n_agents + 63) / 64))) return rc;
  if (!h->pdeg[k])
    if (int rc = dalloc(&h->pdeg[k], h->BN)) return rc;
  a.adj_bits = h->adj_bits[k];
  a.degree_out = h->pdeg[k];
  *bw = k;
  return GF_OK;
}

// Flocking-v0 k nearest with a step (0: none).
//  1: the step also writes this state's adjacency bits and degrees, from which the kNN
//     kernel that follows ranks each agent's neighbours;
//  2: (fe_step, k = 7, no variant) the step ranks them itself, in its feature pass, and
//     the kNN kernel that follows (rim mode) only ranks the rows it could not.
int knn_mode(const fe_handle* h, int flags, bool dyn) {
  if (!(flags & FE_WITH_KNN) || h->cfg.n_neighbors <= 0) return 0;
  const bool variant = h->has_variant || h->dt_per_env;
  if (dyn && gf::step_fused_knn_ok(h->cfg.n_agents, h->R, h->cfg.n_neighbors, variant, h->prefetch != 0)) return 2;
  return 1;
}

// Output buffers of a launch that writes x[xw] (xw < 0: none): picks the bits buffer and
// orders the step streams after the kNN launches still reading what it overwrites.
int prepare_outputs(fe_handle* h, int flags, gf::StepArgs& a, int xw) {
  const int km = knn_mode(h, flags, xw >= 0);
  const bool packed = flags & FE_PACKED_NETWORK;
  int bw = -1;
  if (int rc = packed_outputs(h, packed || km == 1, a, &bw)) return rc;
  if (km == 2) {  // fused selection into the kNN buffers of the state it writes
    const int N = h->cfg.n_agents;
    int jb = 1;
    while ((1 << jb) < N) ++jb;
    a.knn_idx = h->knn_idx[xw];
    a.knn_obs = h->knn_obs[xw];
    a.knn_r2 = h->knn_r2[xw];
    a.knn_rimflag = h->knn_rimflag[xw];
    a.knn_jbits = jb;
    a.knn_qmax = (1u << (32 - jb)) - 2u;  // below the all-ones empty-slot key
    a.knn_qmaxd = static_cast<double>(a.knn_qmax);
    a.knn_qscale = std::ldexp(1.0, 32 - jb);
  }
  if (int rc = wait_knn_readers(h, xw, bw)) return rc;
  if (bw >= 0) h->bits_cur = bw;  // the launch that follows fills it
  if (packed) h->has_packed = true;
  return GF_OK;
}

gf::StepArgs base_args(fe_handle* h) {
  gf::StepArgs a{};
  a.knn_exact = h->knn_exact;
  a.dt = h->cfg.dt;
  a.action_scalar = h->cfg.action_scalar;
  a.cr = h->cfg.comm_radius;
  a.cr2 = h->cfg.comm_radius * h->cfg.comm_radius;
  a.dt_f = static_cast<float>(h->cfg.dt);
  a.as_f = static_cast<float>(h->cfg.action_scalar);
  a.N = h->cfg.n_agents;
  a.B = h->cfg.n_envs;
  a.R = h->R;
  a.T = h->T;
  a.bpe = h->bpe;
  a.mean_pooling = h->cfg.mean_pooling;
  a.centralized = h->cfg.centralized;
  a.diag = h->diag;
  a.prefetch = h->prefetch;
  a.u_scale = h->cfg.action_scalar;
  a.us_f = a.as_f;
  a.x_scale = 1.0;
  if (h->has_variant || h->dt_per_env) {
    a.variant = 1;
    if (h->has_variant) {
      a.n_frozen = h->var.n_frozen;
      a.n_vel_zero = h->var.n_vel_zero;
      a.u_scale = h->var.u_scale;
      a.u_clip = h->var.u_clip;
      a.x_scale = h->var.x_scale;
      a.ctrl_clip = h->var.ctrl_clip;
      a.us_f = static_cast<float>(a.u_scale);
      a.uc_f = static_cast<float>(a.u_clip);
    }
    a.dt_env = h->dt_per_env ? h->dt_env : nullptr;
  }
  return a;
}

// The launch arguments of envs [b0, b0 + nb) of a batched launch a.
gf::StepArgs env_range(const fe_handle* h, const gf::StepArgs& a, int b0, int nb, bool uf64) {
  const int N = a.N;
  const size_t Wn = (N + 63) / 64, e0 = (size_t)b0 * N;
  gf::StepArgs r = a;
  r.B = nb;
  r.x_in = a.x_in + e0 * 4;
  if (a.x_out) r.x_out = a.x_out + e0 * 4;
  if (a.u) r.u = static_cast<const char*>(a.u) + e0 * 2 * (uf64 ? 8 : 4);
  if (a.state_values) r.state_values = a.state_values + e0 * 6;
  if (a.network) r.network = a.network + e0 * N;
  if (a.ctrl_out) r.ctrl_out = a.ctrl_out + e0 * 2;
  if (a.reward) r.reward = a.reward + b0;
  if (a.reward2) r.reward2 = a.reward2 + b0;
  if (a.dt_env) r.dt_env = a.dt_env + b0;
  if (a.adj_bits) r.adj_bits = a.adj_bits + e0 * Wn;
  if (a.degree_out) r.degree_out = a.degree_out + e0;
  if (a.knn_idx) {
    const size_t K = h->cfg.n_neighbors;
    r.knn_idx = a.knn_idx + e0 * K;
    r.knn_obs = a.knn_obs + e0 * 4 * K;
    r.knn_r2 = a.knn_r2 + e0;
    r.knn_rimflag = a.knn_rimflag + (size_t)b0 * ((N + gf::kThreads - 1) / gf::kThreads);
  }
  return r;
}

int timed_launch(fe_handle* h, const gf::StepArgs& a_in, bool dyn, bool uf64, bool ctrl) {
  gf::StepArgs a = a_in;
  a.store_fast = h->store_fast[ctrl ? 1 : 0];
  const bool split = split_next(h, a.B);
  h->other_work = false;
  h->last_b0 = split ? (a.B + 1) / 2 : 0;
  if (split) {
    // two launches: envs [0, B0) on `stream`, [B0, B) on `stream2`, each after its own
    // half of the previous step; stream2 also waits for whatever `stream` was given
    // since (host action copies, state uploads, consumers of the last outputs)
    const int B = a.B, B0 = (B + 1) / 2;
    const gf::StepArgs a1 = env_range(h, a, B0, B - B0, uf64);
    hipError_t e = hipSuccess;
    if (h->dephase && B0 >= 2) {
      // both streams idle (the first split step after other work): the second half
      // would start beside the first and the two would run in phase for many steps.
      // The first half's first quarter goes alone, the second half starts after it, and
      // the rest of the first half runs beside that, so the halves start a quarter
      // period apart.
      const int Bq = B0 / 2;
      e = gf::launch_step(env_range(h, a, 0, Bq, uf64), dyn, uf64, ctrl, h->stream);
      GF_HIP(hipEventRecord(h->ev_main, h->stream));
      GF_HIP(hipStreamWaitEvent(h->stream2, h->ev_main, 0));
      h->main_dirty = h->dephase = false;
      if (e == hipSuccess) e = gf::launch_step(a1, dyn, uf64, ctrl, h->stream2);
      if (e == hipSuccess) e = gf::launch_step(env_range(h, a, Bq, B0 - Bq, uf64), dyn, uf64, ctrl, h->stream);
    } else {
      if (h->main_dirty) {
        GF_HIP(hipEventRecord(h->ev_main, h->stream));
        GF_HIP(hipStreamWaitEvent(h->stream2, h->ev_main, 0));
        h->main_dirty = false;
      }
      e = gf::launch_step(env_range(h, a, 0, B0, uf64), dyn, uf64, ctrl, h->stream);
      if (e == hipSuccess) e = gf::launch_step(a1, dyn, uf64, ctrl, h->stream2);
    }
    if (e != hipSuccess) return fail_hip("flock_step_kernel launch", e);
    h->s2_pending = true;
    if (h->timing) h->tw_steps++;
    return GF_OK;
  }
  if (int rc = join_s2(h)) return rc;  // a single launch covers both halves
  h->main_dirty = h->dephase = true;
  if (h->timing && h->nsplit > 1) h->tw_steps++;  // the window counts every step
  // a sampled launch is bracketed by two events (which also keep it from overlapping
  // its neighbours, so sampling every launch costs the stream ~7 us per step)
  const bool sample = h->timing && (h->timing_count++ % h->timing_stride) == 0;
  if (sample) {
    if (h->ev_used + 2 > h->ev.size()) {
      for (int k = 0; k < 64; ++k) {
        hipEvent_t e;
        GF_HIP(hipEventCreate(&e));
        h->ev.push_back(e);
      }
    }
    GF_HIP(hipEventRecord(h->ev[h->ev_used], h->stream));
  }
  hipError_t e = gf::launch_step(a, dyn, uf64, ctrl, h->stream);
  if (e != hipSuccess) return fail_hip("flock_step_kernel launch", e);
  if (sample) {
    GF_HIP(hipEventRecord(h->ev[h->ev_used + 1], h->stream));
    h->ev_used += 2;
  }
  return GF_OK;
}

// kNN of the current state (mode: knn_mode; 0 = a full kNN with no step behind it):
// 1: the last launch wrote this state's adjacency (packed outputs), which lets agents
// with >= k neighbours rank only those; 2: the last launch ranked the rows it could.
// fin: the drop-in step's completion flag, carried by the (single, unsplit) rim launch
int launch_knn_cur(fe_handle* h, int mode, int32_t* idx_to = nullptr, float* obs_to = nullptr,
                   const gf::DoneFlag* fin = nullptr) {
#ifdef GF_DIAG
  if (mode == 2 && (h->diag & 0x80000)) {  // ablation: no rim kNN launch (timing only)
    h->has_knn = true;
    return GF_OK;
  }
#endif
  auto& r = h->kread[h->cur];
  if (mode == 2 && h->knn_exact) {
    // envs this small: the fused step ranks every row exactly itself (KX), none is left
    // to the rim kernel, so it is not launched
    r.live = false;
    r.bmask = 0;
    h->has_knn = true;
    return GF_OK;
  }
  gf::KnnArgs k{};
  k.x = h->x[h->cur];
  k.adj_bits = mode == 1 ? h->adj_bits[h->bits_cur] : nullptr;
  k.degree = mode == 1 ? h->pdeg[h->bits_cur] : nullptr;
  k.idx = idx_to ? idx_to : h->knn_idx[h->cur];
  k.obs = obs_to ? obs_to : h->knn_obs[h->cur];
  k.rim = mode == 2;
  k.r2k = h->knn_r2[h->cur];
  k.rimflag = h->knn_rimflag[h->cur];
  k.N = h->cfg.n_agents;
  k.B = h->cfg.n_envs;
  k.K = h->cfg.n_neighbors;
  k.diag = (h->diag >> 12) & 0xfc00;  // kNN kernel switches: 0x400000.. -> 0x0400.. (KnnArgs.diag)
  if (mode == 2) {
    // the rim kNN of a fused step goes on the step's own streams, right behind the half
    // that produced its rows: a kNN handle then runs two hardware queues, like a plain
    // one, and the next step's half orders after its rim by stream order (no events)
    if (h->last_b0 > 0 && h->s2_pending && !fin) {
      const int B0 = h->last_b0, N = k.N, K = k.K;
      const size_t e0 = (size_t)B0 * N;
      gf::KnnArgs k1 = k;
      k.B = B0;
      k1.B = h->cfg.n_envs - B0;
      k1.x = k.x + e0 * 4;
      k1.idx = k.idx + e0 * K;
      k1.obs = k.obs + e0 * 4 * K;
      k1.r2k = k.r2k + e0;
      k1.rimflag = k.rimflag + (size_t)B0 * ((N + gf::kThreads - 1) / gf::kThreads);
      k.grid_cap = k1.grid_cap = gf::kKnnRimHalfGrid;
      hipError_t e = gf::launch_knn(k, h->stream);
      if (e == hipSuccess) e = gf::launch_knn(k1, h->stream2);
      if (e != hipSuccess) return fail_hip("flock_knn_kernel launch", e);
    } else {
      if (int rc = join_s2(h)) return rc;
      if (fin) k.fin = *fin;
      hipError_t e = gf::launch_knn(k, h->stream);
      if (e != hipSuccess) return fail_hip("flock_knn_kernel launch", e);
    }
    r.live = false;
    r.bmask = 0;
    h->has_knn = true;
    return GF_OK;
  }
  if (!h->kstream) {  // the separate kNN stream exists only once a full kNN is needed
    hipError_t e = hipStreamCreateWithFlags(&h->kstream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      h->kstream = nullptr;
      return fail_hip("kNN stream create", e);
    }
  }
  // on kstream after everything on both step streams (both halves' state and bits)
  GF_HIP(hipEventRecord(h->ev_kin[0], h->stream));
  GF_HIP(hipStreamWaitEvent(h->kstream, h->ev_kin[0], 0));
  if (h->s2_pending) {
    GF_HIP(hipEventRecord(h->ev_kin[1], h->stream2));
    GF_HIP(hipStreamWaitEvent(h->kstream, h->ev_kin[1], 0));
  }
  hipError_t e = gf::launch_knn(k, h->kstream);
  if (e != hipSuccess) return fail_hip("flock_knn_kernel launch", e);
  GF_HIP(hipEventRecord(r.ev, h->kstream));
  r.live = true;
  if (mode == 1) r.bmask |= 1u << h->bits_cur;
  h->k_pending = true;
  h->has_knn = true;
  return GF_OK;
}

// The kNN radius history describes states the handle no longer holds once the state is
// replaced: forget it (the fused steps then rank neighbours only until it is rebuilt).
hipError_t clear_knn_history(fe_handle* h) {
  for (float* p : h->knn_r2)
    if (p)
      if (hipError_t e = hipMemsetAsync(p, 0, h->BN * sizeof(float), h->stream); e != hipSuccess) return e;
  const size_t nf = (size_t)h->cfg.n_envs * ((h->cfg.n_agents + 255) / 256);
  for (uint8_t* p : h->knn_rimflag)
    if (p)
      if (hipError_t e = hipMemsetAsync(p, 0, nf, h->stream); e != hipSuccess) return e;
  return hipSuccess;
}

int d2h(fe_handle* h, void* dst, const void* src, size_t bytes) {
  GF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, h->stream));
  GF_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

}  // namespace

extern "C" {

const char* fe_last_error(void) { return g_err.c_str(); }
int fe_abi_version(void) { return GF_ABI_VERSION; }

int fe_create(const fe_config* cfg, fe_handle** out) {
  if (!cfg || !out) return fail(GF_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->n_agents < 1 || cfg->n_envs < 1) return fail(GF_EINVAL, "n_agents and n_envs must be >= 1");
  if (cfg->n_neighbors < 0 || cfg->n_neighbors > cfg->n_agents)
    return fail(GF_EINVAL, "n_neighbors must be in [0, n_agents] (the reference indexes argsort columns)");
  if (cfg->n_neighbors > 0) {
    static const int ok[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 16};
    bool found = false;
    for (int k : ok) found |= (k == cfg->n_neighbors);
    if (!found) return fail(GF_EINVAL, "n_neighbors must be one of 1-8, 10, 12, 16");
  }
  if (!(cfg->comm_radius > 0) || !(cfg->action_scalar != 0)) return fail(GF_EINVAL, "bad comm_radius/action_scalar");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(GF_EHIP, "no HIP device available (libgymflock needs an MI355X)");
  if (cfg->device < 0 || cfg->device >= ndev) return fail(GF_EINVAL, "device ordinal out of range");

  fe_handle* h = new fe_handle();
  h->cfg = *cfg;
  const size_t B = cfg->n_envs, N = cfg->n_agents;
  h->BN = B * N;
  h->R = gf::step_rows_per_block(cfg->n_agents);
  h->T = gf::step_tile(cfg->n_agents);
  // a Flocking-v0 handle of one env (the drop-in step) of up to kStepExactKnnMaxOneEnv
  // agents: one tile holds the whole env, which the step then ranks exactly (no keys in the
  // feature pass, no rim kernel)
  if (B == 1 && cfg->n_neighbors > 0 && N <= (size_t)gf::kStepExactKnnMaxOneEnv)
    h->T = static_cast<int>((N + 63) / 64 * 64);
  h->knn_exact = gf::step_knn_exact(cfg->n_agents, h->T, cfg->n_envs) ? 1 : 0;
  // tile loads issued a tile ahead: 1604 -> 1527 us at N=8192 (16 tiles); no gain at 2-8
  // tiles, where its registers cost occupancy instead
  h->prefetch = (cfg->n_agents + h->T - 1) / h->T >= 16 ? 1 : 0;
  // the step + controller uses the plain step's rows per block: with one superset pass 1
  // (kOuter) 32-row blocks beat the 64 of round 3, 169.3 vs 174.4 us at config 2
  // (profiles/r04/ab_ctrl_rows32.txt)
  h->bpe = (cfg->n_agents + h->R - 1) / h->R;
  if ((size_t)h->bpe * B > 0x7fffffff) {
    delete h;
    return fail(GF_EINVAL, "grid too large");
  }
  int rc = GF_OK;
  if ((e = hipSetDevice(cfg->device)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking)) != hipSuccess) {
    release(h);
    return fail_hip("stream create", e);
  }
  if ((rc = dalloc(&h->x[0], h->BN * 4)) || (rc = dalloc(&h->x[1], h->BN * 4)) ||
      (rc = dalloc(reinterpret_cast<double**>(&h->u), h->BN * 2)) || (rc = dalloc(&h->ctrl[0], h->BN * 2)) ||
      (rc = dalloc(&h->ctrl[1], h->BN * 2)) || (rc = dalloc(&h->sv, h->BN * 6)) ||
      (rc = dalloc(&h->net, h->BN * N)) || (rc = dalloc(&h->reward_ring, (size_t)kRewardSlots * B)) ||
      (rc = dalloc(&h->knn_idx[0], h->BN * cfg->n_neighbors)) ||
      (rc = dalloc(&h->knn_idx[1], h->BN * cfg->n_neighbors)) ||
      (rc = dalloc(&h->knn_obs[0], h->BN * 4 * cfg->n_neighbors)) ||
      (rc = dalloc(&h->knn_obs[1], h->BN * 4 * cfg->n_neighbors)) ||
      (cfg->n_neighbors > 0 && ((rc = dalloc(&h->knn_r2[0], h->BN)) || (rc = dalloc(&h->knn_r2[1], h->BN)))) ||
      (cfg->n_neighbors > 0 && ((rc = dalloc(&h->knn_rimflag[0], B * ((N + 255) / 256))) ||
                                (rc = dalloc(&h->knn_rimflag[1], B * ((N + 255) / 256)))))) {
    release(h);
    return rc;
  }
  if ((e = hipEventCreateWithFlags(&h->h2d_ev, hipEventDisableTiming)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&h->stream2, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_s2, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_main, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreate(&h->tw[0])) != hipSuccess || (e = hipEventCreate(&h->tw[1])) != hipSuccess ||
      // no kNN stream here: the fused step's rim kNN runs on the step streams, and a full
      // kNN (fe_get_knn without a step, k != 7, variants) creates one on first use; so a
      // Flocking-v0 handle, like a plain one, runs two streams and two of them fit the
      // process's 4 hardware queues (GPU_MAX_HW_QUEUES)
      (e = hipEventCreateWithFlags(&h->ev_kin[0], hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_kin[1], hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->ev_kjoin, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->kread[0].ev, hipEventDisableTiming)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&h->kread[1].ev, hipEventDisableTiming)) != hipSuccess) {
    release(h);
    return fail_hip("event create", e);
  }
  if ((e = hipMemsetAsync(h->reward_ring, 0, sizeof(double) * kRewardSlots * B, h->stream)) != hipSuccess ||
      (e = clear_knn_history(h)) != hipSuccess ||
      (e = hipStreamSynchronize(h->stream)) != hipSuccess) {
    release(h);
    return fail_hip("init", e);
  }
  *out = h;
  return GF_OK;
}

int fe_destroy(fe_handle* h) {
  release(h);
  return GF_OK;
}

int fe_get_config(const fe_handle* h, fe_config* out) {
  if (!h || !out) return fail(GF_EINVAL, "null argument");
  *out = h->cfg;
  return GF_OK;
}

int fe_set_params(fe_handle* h, const fe_config* cfg) {
  if (!h || !cfg) return fail(GF_EINVAL, "null argument");
  if (cfg->n_agents != h->cfg.n_agents || cfg->n_envs != h->cfg.n_envs || cfg->n_neighbors != h->cfg.n_neighbors ||
      cfg->device != h->cfg.device)
    return fail(GF_EINVAL, "fe_set_params: n_agents, n_envs, n_neighbors and device are fixed at fe_create");
  if (!(cfg->comm_radius > 0) || !(cfg->action_scalar != 0)) return fail(GF_EINVAL, "bad comm_radius/action_scalar");
  // every launch reads these from the handle's config; later steps (after the work already
  // enqueued) use the new values. The kNN radius history was taken under the old radius:
  // forgotten (it only steers which rows the fused step ranks beyond their neighbours)
  if (int rc = use_dev(h)) return rc;
  GF_HIP(clear_knn_history(h));
  // the controls on the device were computed under the old comm_radius / centralized /
  // action_scalar (controller() reads them at call time, :194-226): FE_U_EXPERT and
  // fe_get_controls need a new controller output first
  if (cfg->comm_radius != h->cfg.comm_radius || cfg->centralized != h->cfg.centralized ||
      cfg->action_scalar != h->cfg.action_scalar)
    h->has_ctrl = false;
  h->cfg.comm_radius = cfg->comm_radius;
  h->cfg.dt = cfg->dt;
  h->cfg.action_scalar = cfg->action_scalar;
  h->cfg.mean_pooling = cfg->mean_pooling;
  h->cfg.centralized = cfg->centralized;
  return GF_OK;
}

int fe_set_state(fe_handle* h, const double* x) {
  if (!h || !x) return fail(GF_EINVAL, "null argument");
  if (int rc = use_dev(h)) return rc;
  GF_HIP(hipMemcpyAsync(h->x[h->cur], x, h->BN * 4 * sizeof(double), hipMemcpyHostToDevice, h->stream));
  GF_HIP(clear_knn_history(h));
  GF_HIP(hipStreamSynchronize(h->stream));
  h->has_state = true;
  h->has_ctrl = h->has_obs = h->has_knn = false;
  return GF_OK;
}

int fe_reset_synthetic(fe_handle* h, uint64_t seed, double v_max) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (seed + (uint64_t)h->cfg.n_envs > 0x100000000ull) return fail(GF_EINVAL, "seed + n_envs must fit in 32 bits");
  const int N = h->cfg.n_agents, B = h->cfg.n_envs;
  std::vector<double> x((size_t)B * N * 4);
  const double r_max = std::sqrt(static_cast<double>(N));
  for (int b = 0; b < B; ++b) {
    std::mt19937 mt(static_cast<uint32_t>(seed + b));  // RandomState(seed + b): init_genrand
    auto uniform = [&](double lo, double hi) {          // random_sample (53-bit), then lo + (hi-lo)*u
      const uint32_t a = mt() >> 5, c = mt() >> 6;
      return lo + (hi - lo) * ((a * 67108864.0 + c) / 9007199254740992.0);
    };
    double* e = x.data() + (size_t)b * N * 4;
    std::vector<double> len(N);
    for (int i = 0; i < N; ++i) len[i] = std::sqrt(uniform(0.0, r_max));
    for (int i = 0; i < N; ++i) {
      const double ang = M_PI * uniform(0.0, 2.0);
      e[4 * i] = len[i] * std::cos(ang);
      e[4 * i + 1] = len[i] * std::sin(ang);
    }
    const double b0 = uniform(-v_max, v_max), b1 = uniform(-v_max, v_max);
    for (int i = 0; i < N; ++i) e[4 * i + 2] = uniform(-v_max, v_max) + b0;
    for (int i = 0; i < N; ++i) e[4 * i + 3] = uniform(-v_max, v_max) + b1;
  }
  return fe_set_state(h, x.data());
}

int fe_set_state_env(fe_handle* h, int env, const double* x) {
  if (!h || !x || env < 0) return fail(GF_EINVAL, "bad argument");
  if (int rc = check_env(h, env)) return rc;
  if (int rc = use_dev(h)) return rc;
  const size_t n = (size_t)h->cfg.n_agents * 4;
  GF_HIP(hipMemcpyAsync(h->x[h->cur] + env * n, x, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
  GF_HIP(clear_knn_history(h));
  GF_HIP(hipStreamSynchronize(h->stream));
  h->has_state = true;
  h->has_ctrl = h->has_obs = h->has_knn = false;
  return GF_OK;
}

int fe_get_state(fe_handle* h, double* x) {
  if (!h || !x) return fail(GF_EINVAL, "null argument");
  if (!h->has_state) return fail(GF_ESTATE, "state not set");
  if (int rc = use_dev(h)) return rc;
  return d2h(h, x, h->x[h->cur], h->BN * 4 * sizeof(double));
}

int fe_get_state_env(fe_handle* h, int env, double* x) {
  if (!h || !x || env < 0) return fail(GF_EINVAL, "bad argument");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_state) return fail(GF_ESTATE, "state not set");
  if (int rc = use_dev(h)) return rc;
  const size_t n = (size_t)h->cfg.n_agents * 4;
  return d2h(h, x, h->x[h->cur] + env * n, n * sizeof(double));
}

int fe_compute_helpers(fe_handle* h, int flags) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->has_state) return fail(GF_ESTATE, "state not set");
  if (int rc = use_dev_step(h)) return rc;
  const bool ctrl = flags & FE_WITH_CONTROLLER;
  if (int rc = next_reward_slot(h)) return rc;
  gf::StepArgs a = base_args(h);
  a.x_in = h->x[h->cur];
  a.state_values = (flags & FE_NO_STATE_VALUES) ? nullptr : h->sv;
  a.network = (flags & FE_NO_NETWORK) ? nullptr : h->net;
  a.ctrl_out = ctrl ? h->ctrl[h->ccur ^ 1] : nullptr;
  a.reward = cur_reward(h);
  const int km = knn_mode(h, flags, false);
  if (int rc = prepare_outputs(h, flags, a, -1)) return rc;
  if (int rc = timed_launch(h, a, false, false, ctrl)) return rc;
  if (ctrl) {
    h->ccur ^= 1;
    h->has_ctrl = true;
  }
  h->has_obs = true;
  h->obs_on_host = false;
  if (km)
    if (int rc = launch_knn_cur(h, km)) return rc;
  return GF_OK;
}

}  // extern "C"

namespace {
// The host-action copy stream and its two device buffers (fe_handle::ustream), on first use.
int ensure_ucopy(fe_handle* h) {
  if (h->ustream) return GF_OK;
  for (int k = 0; k < 2; ++k) {
    if (int rc = dalloc(reinterpret_cast<double**>(&h->ubuf[k]), h->BN * 2)) return rc;
    GF_HIP(hipEventCreateWithFlags(&h->ev_ucopy[k], hipEventDisableTiming));
    GF_HIP(hipEventCreateWithFlags(&h->ev_uread[k][0], hipEventDisableTiming));
    GF_HIP(hipEventCreateWithFlags(&h->ev_uread[k][1], hipEventDisableTiming));
  }
  GF_HIP(hipStreamCreateWithFlags(&h->ustream, hipStreamNonBlocking));
  return GF_OK;
}
}  // namespace

extern "C" {

int fe_step(fe_handle* h, const void* u, int flags) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->has_state) return fail(GF_ESTATE, "state not set (call fe_set_state first)");
  if (int rc = use_dev_step(h)) return rc;
  const bool ctrl = flags & FE_WITH_CONTROLLER;
  bool uf64 = flags & FE_U_F64;
  const void* up = nullptr;
  int uk = -1;  // the action buffer of a split step's host actions (ubuf), or none
  if (flags & FE_U_EXPERT) {
    if (!h->has_ctrl) return fail(GF_ESTATE, "FE_U_EXPERT needs a previous controller output");
    up = h->ctrl[h->ccur];
    uf64 = true;
  } else if (flags & FE_U_RESIDENT) {
    if (h->u_resident_f64 < 0) return fail(GF_ESTATE, "FE_U_RESIDENT needs fe_set_actions first");
    up = h->u;
    uf64 = h->u_resident_f64 == 1;
  } else if (!u) {
    return fail(GF_EINVAL, "null action pointer");
  } else if (flags & FE_U_DEVICE) {
    // the caller may have written the actions on the handle's stream (fe_buffers.stream):
    // the second half's stream waits for it (an event, no host sync); the halves keep
    // their phase (no de-phasing: that is for the first split step after other work)
    up = u;
    h->main_dirty = true;
  } else if (split_next(h, h->cfg.n_envs)) {
    // a split step: the copy on the action stream, overlapping the step before
    if (int rc = ensure_ucopy(h)) return rc;
    uk = h->ucur;
    h->ucur ^= 1;
    if (h->uread_live[uk]) {  // both halves of the step that read this buffer
      GF_HIP(hipStreamWaitEvent(h->ustream, h->ev_uread[uk][0], 0));
      GF_HIP(hipStreamWaitEvent(h->ustream, h->ev_uread[uk][1], 0));
    }
    GF_HIP(hipMemcpyAsync(h->ubuf[uk], u, h->BN * 2 * (uf64 ? 8 : 4), hipMemcpyHostToDevice, h->ustream));
    GF_HIP(hipEventRecord(h->ev_ucopy[uk], h->ustream));
    GF_HIP(hipStreamWaitEvent(h->stream, h->ev_ucopy[uk], 0));
    GF_HIP(hipStreamWaitEvent(h->stream2, h->ev_ucopy[uk], 0));
    up = h->ubuf[uk];
  } else {
    // the previous step's second half may still read h->u: copy after it
    if (int rc = join_s2(h)) return rc;
    GF_HIP(hipMemcpyAsync(h->u, u, h->BN * 2 * (uf64 ? 8 : 4), hipMemcpyHostToDevice, h->stream));
    GF_HIP(hipEventRecord(h->h2d_ev, h->stream));
    h->main_dirty = h->other_work = true;
    up = h->u;
    h->u_resident_f64 = -1;  // the buffer now holds this call's actions
  }
  if (int rc = next_reward_slot(h)) return rc;
  gf::StepArgs a = base_args(h);
  a.x_in = h->x[h->cur];
  a.x_out = h->x[h->cur ^ 1];
  a.u = up;
  a.state_values = (flags & FE_NO_STATE_VALUES) ? nullptr : h->sv;
  a.network = (flags & FE_NO_NETWORK) ? nullptr : h->net;
  a.ctrl_out = ctrl ? h->ctrl[h->ccur ^ 1] : nullptr;
  a.reward = cur_reward(h);
  const int km = knn_mode(h, flags, true);
  if (int rc = prepare_outputs(h, flags, a, h->cur ^ 1)) return rc;
  if (int rc = timed_launch(h, a, true, uf64, ctrl)) return rc;
  if (uk >= 0) {  // the halves that read the buffer: the copy two calls on waits for them
    GF_HIP(hipEventRecord(h->ev_uread[uk][0], h->stream));
    GF_HIP(hipEventRecord(h->ev_uread[uk][1], h->last_b0 ? h->stream2 : h->stream));
    h->uread_live[uk] = true;
  }
  h->cur ^= 1;
  if (ctrl) h->ccur ^= 1;
  h->has_ctrl = ctrl;
  h->has_obs = true;
  h->obs_on_host = false;
  h->has_knn = false;
  if (km)
    if (int rc = launch_knn_cur(h, km)) return rc;
  // the host action buffer is borrowed only for this call: wait for its copy, not the step
  if (uk >= 0) GF_HIP(hipEventSynchronize(h->ev_ucopy[uk]));
  else if (!(flags & (FE_U_DEVICE | FE_U_EXPERT | FE_U_RESIDENT))) GF_HIP(hipEventSynchronize(h->h2d_ev));
  return GF_OK;
}

// fe_step_host and fe_step_host_knn: knn_idx / knn_obs (either non-NULL) also rank the new
// state's k nearest (the fused selection, or the kNN kernel) and bring them back.
static int step_host_impl(fe_handle* h, const void* u, float* state_values, float* network, double* rewards,
                          double* controls, int32_t* knn_idx, float* knn_obs, int flags) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->has_state) return fail(GF_ESTATE, "state not set (call fe_set_state first)");
  if (flags & ~(FE_U_F64 | FE_WITH_CONTROLLER)) return fail(GF_EINVAL, "flags: FE_U_F64 and FE_WITH_CONTROLLER only");
  const bool knn = knn_idx || knn_obs;
  if (knn && h->cfg.n_neighbors <= 0) return fail(GF_EINVAL, "handle created with n_neighbors = 0");
  if (controls) flags |= FE_WITH_CONTROLLER;
  // one launch on the handle's stream, after all of its outstanding work
  if (int rc = use_dev(h)) return rc;
  const bool dyn = u != nullptr, ctrl = flags & FE_WITH_CONTROLLER, uf64 = dyn && (flags & FE_U_F64);
  const void* up = nullptr;
  // one env of one tile: the actions travel in the kernel arguments (no read over the
  // link inside the kernel); otherwise page-locked actions are read in place, others
  // copied to the device first
  // (the fused kNN step with the controller has an inline-actions form only for envs
  // ranked exactly in the step, gf::step_knn_exact)
  const bool uin = dyn && !(knn && ctrl && !h->knn_exact) && h->cfg.n_envs == 1 && h->cfg.n_agents <= h->T && !h->has_variant && !h->dt_per_env &&
                   h->BN * 2 * (uf64 ? 8 : 4) <= (size_t)gf::kUInlineBytes;
  if (uin) {
    up = u;
  } else if (dyn) {
    up = mapped_ptr(const_cast<void*>(u));  // page-locked: the kernel reads it in place
    if (!up) {
      GF_HIP(hipMemcpyAsync(h->u, u, h->BN * 2 * (uf64 ? 8 : 4), hipMemcpyHostToDevice, h->stream));
      up = h->u;
      h->u_resident_f64 = -1;
    }
  }
  if (int rc = next_reward_slot(h)) return rc;
  // page-locked destinations are written by the kernel through their mapped addresses;
  // others get the device buffer and a copy after the launch
  float* sv_m = state_values ? static_cast<float*>(mapped_ptr(state_values)) : nullptr;
  float* net_m = network ? static_cast<float*>(mapped_ptr(network)) : nullptr;
  double* rw_m = rewards ? static_cast<double*>(mapped_ptr(rewards)) : nullptr;
  double* ct_m = controls ? static_cast<double*>(mapped_ptr(controls)) : nullptr;
  gf::StepArgs a = base_args(h);
  a.x_in = h->x[h->cur];
  if (dyn) {
    a.x_out = h->x[h->cur ^ 1];
    a.u = up;
    a.u_inline = uin ? 1 : 0;
  }
  a.state_values = state_values ? (sv_m ? sv_m : h->sv) : nullptr;
  a.network = network ? (net_m ? net_m : h->net) : nullptr;
  a.ctrl_out = ctrl ? (ct_m ? ct_m : h->ctrl[h->ccur ^ 1]) : nullptr;
  a.reward = cur_reward(h);
  a.reward2 = rw_m;
  const int kflags = knn ? FE_WITH_KNN : 0, km = knn_mode(h, kflags, dyn);
  if (int rc = prepare_outputs(h, kflags, a, dyn ? h->cur ^ 1 : -1)) return rc;
  // fused selection with both destinations page-locked: the step and its rim kNN write
  // the rows straight into them (the device's kNN buffers of this state are then not
  // written: fe_get_knn recomputes them if asked)
  int32_t* idx_m = knn_idx ? static_cast<int32_t*>(mapped_ptr(knn_idx)) : nullptr;
  float* obs_m = knn_obs ? static_cast<float*>(mapped_ptr(knn_obs)) : nullptr;
  const bool kdirect = km == 2 && idx_m && obs_m;
  if (kdirect) {
    a.knn_idx = idx_m;
    a.knn_obs = obs_m;
  }
  // When the call's device work ends with one launch that writes the last outputs to
  // page-locked memory (every output page-locked, no copy after it: the step, or the rim
  // kNN behind it), the host waits for that kernel's own completion flag, not for the
  // stream (done_flag.h: ~8 us sooner)
  const bool rim_last = knn && !h->knn_exact;
  // (diagnostic build: the ablation that skips the rim kNN launch would drop the flag it
  // carries; the host then waits for the stream)
  const bool fin = (!state_values || sv_m) && (!network || net_m) && (!rewards || rw_m) && (!ctrl || ct_m) &&
                   (!knn || kdirect) && !(rim_last && (h->diag & 0x80000));
  gf::DoneFlag fd{};
  if (fin) {
    if (!h->fin_cnt) {
      if (int rc = dalloc(&h->fin_cnt, 1)) return rc;
      GF_HIP(hipMemsetAsync(h->fin_cnt, 0, sizeof(int32_t), h->stream));
      void* p = nullptr;
      GF_HIP(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
      h->fin_host = static_cast<int32_t*>(p);
      *h->fin_host = 0;
      h->fin_dev = static_cast<int32_t*>(mapped_ptr(p));
      if (!h->fin_dev) return fail(GF_EHIP, "completion flag: no mapped address");
    }
    fd.cnt = h->fin_cnt;
    fd.host = h->fin_dev;
    h->fin_seq = (h->fin_seq & 0x3fffffff) + 1;  // never 0 (the word's initial value), no overflow
    fd.seq = h->fin_seq;
    if (!rim_last) a.fin = fd;
    else a.fin.fence = 1;  // the step's page-locked writes land before the rim kNN's flag
  }
  if (int rc = timed_launch(h, a, dyn, uf64, ctrl)) return rc;
  if (dyn) h->cur ^= 1;
  const size_t nsv = h->BN * 6, nnet = h->BN * (size_t)h->cfg.n_agents, nct = h->BN * 2;
  if (state_values && !sv_m)
    GF_HIP(hipMemcpyAsync(state_values, h->sv, nsv * 4, hipMemcpyDeviceToHost, h->stream));
  if (network && !net_m) GF_HIP(hipMemcpyAsync(network, h->net, nnet * 4, hipMemcpyDeviceToHost, h->stream));
  if (rewards && !rw_m)
    GF_HIP(hipMemcpyAsync(rewards, cur_reward(h), (size_t)h->cfg.n_envs * 8, hipMemcpyDeviceToHost, h->stream));
  if (ctrl && !ct_m) {
    h->ccur ^= 1;
    if (controls) GF_HIP(hipMemcpyAsync(controls, h->ctrl[h->ccur], nct * 8, hipMemcpyDeviceToHost, h->stream));
  }
  if (dyn || ctrl) h->has_ctrl = ctrl && !ct_m;  // device controls of the current state
  h->has_obs = true;
  h->obs_on_host = sv_m || net_m;
  h->has_knn = false;
  if (knn) {
    // the rim (or whole) kNN of the new state, then its rows to the host: page-locked
    // destinations by one copy kernel through their mapped addresses (a DMA copy costs
    // ~12 us of latency each), others by copies
    if (int rc = launch_knn_cur(h, km, kdirect ? idx_m : nullptr, kdirect ? obs_m : nullptr,
                                (fin && rim_last) ? &fd : nullptr))
      return rc;
    if (int rc = join_s2(h)) return rc;
    if (int rc = join_k(h)) return rc;
    if (kdirect) {
      h->has_knn = false;
      knn_idx = nullptr;
      knn_obs = nullptr;
    }
    const size_t nk = h->BN * (size_t)h->cfg.n_neighbors;
    OutCopy c{};
    c.src[0] = reinterpret_cast<const float*>(h->knn_idx[h->cur]);
    c.src[1] = h->knn_obs[h->cur];
    c.n[0] = nk;
    c.n[1] = 4 * nk;
    if (knn_idx && (c.dst[0] = static_cast<float*>(mapped_ptr(knn_idx)))) knn_idx = nullptr;
    if (knn_obs && (c.dst[1] = static_cast<float*>(mapped_ptr(knn_obs)))) knn_obs = nullptr;
    if (c.dst[0] || c.dst[1]) {
      const int grid = static_cast<int>(std::min<size_t>((nk + 255) / 256, 1024));
      hipLaunchKernelGGL(out_copy_kernel, dim3(grid), dim3(256), 0, h->stream, c);
      GF_HIP(hipGetLastError());
    }
    if (knn_idx) GF_HIP(hipMemcpyAsync(knn_idx, h->knn_idx[h->cur], nk * 4, hipMemcpyDeviceToHost, h->stream));
    if (knn_obs) GF_HIP(hipMemcpyAsync(knn_obs, h->knn_obs[h->cur], nk * 16, hipMemcpyDeviceToHost, h->stream));
  }
  if (fin) {
    const hipError_t q = gf::wait_done(h->fin_host, h->fin_seq, h->stream);
    if (q == hipErrorUnknown) return fail(GF_EHIP, "fe_step_host: the step finished without its completion flag");
    if (q != hipSuccess) return fail_hip("fe_step_host", q);
    return GF_OK;
  }
  // spin on the stream: the drop-in step is latency-bound (tens of us), and a blocking
  // wait's wake-up costs a sizeable part of that
  for (;;) {
    const hipError_t q = hipStreamQuery(h->stream);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) return fail_hip("fe_step_host", q);
  }
  return GF_OK;
}

int fe_step_host(fe_handle* h, const void* u, float* state_values, float* network, double* rewards,
                 double* controls, int flags) {
  return step_host_impl(h, u, state_values, network, rewards, controls, nullptr, nullptr, flags);
}

int fe_step_host_knn(fe_handle* h, const void* u, float* state_values, float* network, double* rewards,
                     int32_t* knn_idx, float* knn_obs, int flags) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!knn_idx && !knn_obs) return fail(GF_EINVAL, "knn_idx and knn_obs both NULL (use fe_step_host)");
  return step_host_impl(h, u, state_values, network, rewards, nullptr, knn_idx, knn_obs, flags);
}

int fe_step_host_knn_ctrl(fe_handle* h, const void* u, float* state_values, float* network, double* rewards,
                          double* controls, int32_t* knn_idx, float* knn_obs, int flags) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!knn_idx && !knn_obs) return fail(GF_EINVAL, "knn_idx and knn_obs both NULL (use fe_step_host)");
  return step_host_impl(h, u, state_values, network, rewards, controls, knn_idx, knn_obs, flags);
}

int fe_set_variant(fe_handle* h, const fe_variant* v) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!v) {
    h->has_variant = false;
    return GF_OK;
  }
  if (v->n_frozen < 0 || v->n_vel_zero < 0) return fail(GF_EINVAL, "negative agent count");
  if (!(v->x_scale != 0.0) || !std::isfinite(v->x_scale) || !std::isfinite(v->u_scale))
    return fail(GF_EINVAL, "x_scale must be finite and non-zero, u_scale finite");
  h->var = *v;
  h->has_variant = true;
  return GF_OK;
}

int fe_set_dt(fe_handle* h, const double* dt) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!dt) {
    h->dt_per_env = false;
    return GF_OK;
  }
  if (int rc = use_dev(h)) return rc;
  if (!h->dt_env)
    if (int rc = dalloc(&h->dt_env, (size_t)h->cfg.n_envs)) return rc;
  GF_HIP(hipMemcpyAsync(h->dt_env, dt, (size_t)h->cfg.n_envs * sizeof(double), hipMemcpyHostToDevice, h->stream));
  GF_HIP(hipStreamSynchronize(h->stream));
  h->dt_per_env = true;
  return GF_OK;
}

int fe_set_actions(fe_handle* h, const void* u, int f64) {
  if (!h || !u) return fail(GF_EINVAL, "null argument");
  if (int rc = use_dev(h)) return rc;
  GF_HIP(hipMemcpyAsync(h->u, u, h->BN * 2 * (f64 ? 8 : 4), hipMemcpyHostToDevice, h->stream));
  GF_HIP(hipStreamSynchronize(h->stream));
  h->u_resident_f64 = f64 ? 1 : 0;
  return GF_OK;
}

int fe_controller(fe_handle* h, int centralized, double* u_out) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->has_state) return fail(GF_ESTATE, "state not set");
  if (int rc = use_dev(h)) return rc;
  gf::StepArgs a = base_args(h);
  if (centralized >= 0) a.centralized = centralized ? 1 : 0;
  a.x_in = h->x[h->cur];
  a.ctrl_out = h->ctrl[h->ccur ^ 1];
  hipError_t e = gf::launch_step(a, false, false, true, h->stream);
  if (e != hipSuccess) return fail_hip("controller launch", e);
  h->ccur ^= 1;
  h->has_ctrl = true;
  if (u_out) return d2h(h, u_out, h->ctrl[h->ccur], h->BN * 2 * sizeof(double));
  return GF_OK;
}

int fe_get_stats(fe_handle* h, int env, double* vel_diffs, double* min_dists) {
  return fe_get_stats_ex(h, env, vel_diffs, min_dists, nullptr);
}

int fe_get_stats_ex(fe_handle* h, int env, double* vel_diffs, double* min_dists, int32_t* degree) {
  if (!h || env < 0) return fail(GF_EINVAL, "bad argument");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_state) return fail(GF_ESTATE, "state not set");
  if (int rc = use_dev(h)) return rc;
  if (!h->vel_diffs) {
    if (int rc = dalloc(&h->vel_diffs, h->BN)) return rc;
    if (int rc = dalloc(&h->min_dists, h->BN)) return rc;
    if (int rc = dalloc(&h->degree, h->BN)) return rc;
  }
  gf::StatsArgs s{h->x[h->cur], h->vel_diffs, h->min_dists, h->degree,
                  h->cfg.comm_radius * h->cfg.comm_radius, h->cfg.n_agents, h->cfg.n_envs};
  hipError_t e = gf::launch_stats(s, h->stream);
  if (e != hipSuccess) return fail_hip("stats launch", e);
  const size_t N = h->cfg.n_agents;
  if (vel_diffs) GF_HIP(hipMemcpyAsync(vel_diffs, h->vel_diffs + env * N, N * 8, hipMemcpyDeviceToHost, h->stream));
  if (min_dists) GF_HIP(hipMemcpyAsync(min_dists, h->min_dists + env * N, N * 8, hipMemcpyDeviceToHost, h->stream));
  if (degree) GF_HIP(hipMemcpyAsync(degree, h->degree + env * N, N * 4, hipMemcpyDeviceToHost, h->stream));
  GF_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

namespace {
// get_stats (:136-143) on every env of the current state, then each env's means of the
// two arrays into stats_sum (B,2), on the handle's stream. A pending stats gather's
// staging copy may still read stats_sum: the host waits for that gather (bounded, as
// next_reward_slot; on expiry the metrics path is torn down and the summary goes on).
int stats_summary_dev(fe_handle* h) {
  if (!h->vel_diffs) {
    if (int rc = dalloc(&h->vel_diffs, h->BN)) return rc;
    if (int rc = dalloc(&h->min_dists, h->BN)) return rc;
    if (int rc = dalloc(&h->degree, h->BN)) return rc;
  }
  if (!h->stats_sum)
    if (int rc = dalloc(&h->stats_sum, (size_t)h->cfg.n_envs * 2)) return rc;
  if (h->sg_pending && h->comm && !stage_complete(h, kWordStatsCopy, h->stage_seq[kWordStatsCopy])) {
    const int rc = stage_wait(h, kWordStatsCopy, h->stage_seq[kWordStatsCopy], "stats all-gather (send block reuse)");
    if (rc == GF_ECOMM) h->comm_lost = g_err;  // torn down: the summary goes on
    else if (rc != GF_OK) return rc;
  }
  gf::StatsArgs s{h->x[h->cur], h->vel_diffs, h->min_dists, h->degree,
                  h->cfg.comm_radius * h->cfg.comm_radius, h->cfg.n_agents, h->cfg.n_envs};
  hipError_t e = gf::launch_stats(s, h->stream);
  if (e == hipSuccess) e = gf::launch_stats_summary(s, h->stats_sum, h->stream);
  if (e != hipSuccess) return fail_hip("stats launch", e);
  return GF_OK;
}
}  // namespace

int fe_stats_summary(fe_handle* h, double* dst) {
  if (!h || !dst) return fail(GF_EINVAL, "null argument");
  if (!h->has_state) return fail(GF_ESTATE, "state not set");
  if (int rc = use_dev(h)) return rc;
  if (int rc = stats_summary_dev(h)) return rc;
  return d2h(h, dst, h->stats_sum, (size_t)h->cfg.n_envs * 2 * sizeof(double));
}

int fe_get_state_values(fe_handle* h, int env, float* dst) {
  if (!h || !dst) return fail(GF_EINVAL, "null argument");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_obs) return fail(GF_ESTATE, "no observation computed yet");
  if (h->obs_on_host) return fail(GF_ESTATE, "the last step wrote its observations to host arrays (fe_step_host)");
  if (int rc = use_dev(h)) return rc;
  const size_t n = (size_t)h->cfg.n_agents * 6;
  return env < 0 ? d2h(h, dst, h->sv, h->BN * 6 * 4) : d2h(h, dst, h->sv + env * n, n * 4);
}

int fe_get_network(fe_handle* h, int env, float* dst) {
  if (!h || !dst) return fail(GF_EINVAL, "null argument");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_obs) return fail(GF_ESTATE, "no observation computed yet");
  if (h->obs_on_host) return fail(GF_ESTATE, "the last step wrote its observations to host arrays (fe_step_host)");
  if (int rc = use_dev(h)) return rc;
  const size_t n = (size_t)h->cfg.n_agents * h->cfg.n_agents;
  return env < 0 ? d2h(h, dst, h->net, h->BN * h->cfg.n_agents * 4) : d2h(h, dst, h->net + env * n, n * 4);
}

int fe_get_network_rows(fe_handle* h, int env, int row0, int nrows, float* dst) {
  if (!h || !dst || env < 0 || row0 < 0 || nrows < 0 || row0 + nrows > h->cfg.n_agents)
    return fail(GF_EINVAL, "bad argument");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_obs || h->obs_on_host) return fail(GF_ESTATE, "no device observation (none yet, or fe_step_host wrote it to host arrays)");
  if (int rc = use_dev(h)) return rc;
  const size_t N = h->cfg.n_agents;
  return d2h(h, dst, h->net + (env * N + row0) * N, (size_t)nrows * N * 4);
}

int fe_get_network_packed(fe_handle* h, int env, uint64_t* bits, int32_t* degree) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_packed) return fail(GF_ESTATE, "no FE_PACKED_NETWORK step yet");
  if (int rc = use_dev(h)) return rc;
  const size_t N = h->cfg.n_agents, Wn = (N + 63) / 64;
  if (bits) {
    const size_t n = N * Wn;
    const uint64_t* src = h->adj_bits[h->bits_cur];
    if (int rc = env < 0 ? d2h(h, bits, src, h->BN * Wn * 8) : d2h(h, bits, src + env * n, n * 8)) return rc;
  }
  if (degree) {
    const int32_t* src = h->pdeg[h->bits_cur];
    if (int rc = env < 0 ? d2h(h, degree, src, h->BN * 4) : d2h(h, degree, src + env * N, N * 4)) return rc;
  }
  return GF_OK;
}

int fe_get_controls(fe_handle* h, int env, double* dst) {
  if (!h || !dst) return fail(GF_EINVAL, "null argument");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_ctrl) return fail(GF_ESTATE, "no controller output");
  if (int rc = use_dev(h)) return rc;
  const size_t n = (size_t)h->cfg.n_agents * 2;
  const double* src = h->ctrl[h->ccur];
  return env < 0 ? d2h(h, dst, src, h->BN * 2 * 8) : d2h(h, dst, src + env * n, n * 8);
}

int fe_get_outputs(fe_handle* h, int env, float* state_values, float* network, double* rewards, int flags) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (flags & ~FE_OUT_MAPPED) return fail(GF_EINVAL, "flags: 0 or FE_OUT_MAPPED");
  if (int rc = check_env(h, env)) return rc;
  if (!h->has_obs) return fail(GF_ESTATE, "no observation computed yet");
  if (h->obs_on_host && (state_values || network))
    return fail(GF_ESTATE, "the last step wrote its observations to host arrays (fe_step_host)");
  if (int rc = use_dev(h)) return rc;
  const size_t N = h->cfg.n_agents;
  const size_t nsv = env < 0 ? h->BN * 6 : N * 6, nnet = env < 0 ? h->BN * N : N * N;
  if (flags & FE_OUT_MAPPED) {
    // page-locked destinations by one copy kernel; any other one by its own copy below
    OutCopy c{};
    c.src[0] = h->sv + (env < 0 ? 0 : env * N * 6);
    c.src[1] = h->net + (env < 0 ? 0 : env * N * N);
    c.n[0] = nsv;
    c.n[1] = nnet;
    c.rsrc = cur_reward(h);
    c.nr = h->cfg.n_envs;
    if (state_values && (c.dst[0] = static_cast<float*>(mapped_ptr(state_values)))) state_values = nullptr;
    if (network && (c.dst[1] = static_cast<float*>(mapped_ptr(network)))) network = nullptr;
    if (rewards && (c.rdst = static_cast<double*>(mapped_ptr(rewards)))) rewards = nullptr;
    if (c.dst[0] || c.dst[1] || c.rdst) {
      const size_t most = std::max(c.dst[0] ? nsv : 0, c.dst[1] ? nnet : 0) / 4 + 1;
      const int grid = static_cast<int>(std::min<size_t>((most + 255) / 256, 1024));
      hipLaunchKernelGGL(out_copy_kernel, dim3(grid), dim3(256), 0, h->stream, c);
      GF_HIP(hipGetLastError());
    }
  }
  if (rewards)
    GF_HIP(hipMemcpyAsync(rewards, cur_reward(h), (size_t)h->cfg.n_envs * 8, hipMemcpyDeviceToHost, h->stream));
  if (state_values)
    GF_HIP(hipMemcpyAsync(state_values, h->sv + (env < 0 ? 0 : env * N * 6), nsv * 4, hipMemcpyDeviceToHost,
                          h->stream));
  if (network)
    GF_HIP(hipMemcpyAsync(network, h->net + (env < 0 ? 0 : env * N * N), nnet * 4, hipMemcpyDeviceToHost, h->stream));
  GF_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int fe_host_alloc(size_t bytes, void** out) {
  if (!out || bytes == 0) return fail(GF_EINVAL, "bad argument");
  *out = nullptr;
  hipError_t e = hipHostMalloc(out, bytes, hipHostMallocMapped);
  if (e != hipSuccess) {
    *out = nullptr;
    return fail(GF_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
  }
  return GF_OK;
}

int fe_host_free(void* p) {
  if (p) GF_HIP(hipHostFree(p));
  return GF_OK;
}

int fe_get_rewards(fe_handle* h, double* dst) {
  if (!h || !dst) return fail(GF_EINVAL, "null argument");
  if (!h->has_obs) return fail(GF_ESTATE, "no step computed yet");
  if (int rc = use_dev(h)) return rc;
  return d2h(h, dst, cur_reward(h), (size_t)h->cfg.n_envs * 8);
}

int fe_get_knn(fe_handle* h, int env, int32_t* idx, float* obs) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (int rc = check_env(h, env)) return rc;
  if (h->cfg.n_neighbors <= 0) return fail(GF_EINVAL, "handle created with n_neighbors = 0");
  if (int rc = use_dev(h)) return rc;
  if (!h->has_knn) {
    if (!h->has_state) return fail(GF_ESTATE, "state not set");
    if (int rc = launch_knn_cur(h, 0)) return rc;  // no adjacency of this state at hand
    if (int rc = join_k(h)) return rc;               // the copies below read its outputs
  }
  const size_t K = h->cfg.n_neighbors, N = h->cfg.n_agents;
  const size_t off = env < 0 ? 0 : env * N;
  const size_t cnt = env < 0 ? h->BN : N;
  const int32_t* kidx = h->knn_idx[h->cur];
  const float* kobs = h->knn_obs[h->cur];
  if (idx) GF_HIP(hipMemcpyAsync(idx, kidx + off * K, cnt * K * 4, hipMemcpyDeviceToHost, h->stream));
  if (obs) GF_HIP(hipMemcpyAsync(obs, kobs + off * 4 * K, cnt * 4 * K * 4, hipMemcpyDeviceToHost, h->stream));
  GF_HIP(hipStreamSynchronize(h->stream));
  return GF_OK;
}

int fe_device_buffers(fe_handle* h, fe_buffers* out) {
  if (!h || !out) return fail(GF_EINVAL, "null argument");
  // a reader on out->stream sees whole steps (both halves), and the next split step's
  // second half waits for what the caller enqueues there
  if (int rc = use_dev(h)) return rc;
  out->x = h->x[h->cur];
  // fe_step_host wrote the last observation to host arrays only: the device copies are
  // stale, so they are not handed out
  out->state_values = h->obs_on_host ? nullptr : h->sv;
  out->network = h->obs_on_host ? nullptr : h->net;
  out->controls = h->ctrl[h->ccur];
  out->rewards = cur_reward(h);
  out->knn_idx = h->knn_idx[h->cur];  // the current state's (they alternate with the state)
  out->knn_obs = h->knn_obs[h->cur];
  out->stream = h->stream;
  out->adj_bits = h->adj_bits[h->bits_cur];
  out->degree = h->pdeg[h->bits_cur];
  return GF_OK;
}

int fe_sync(fe_handle* h) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (int rc = use_dev(h)) return rc;
  GF_HIP(hipStreamSynchronize(h->stream));
  if (h->comm && !comm_stream_drained(h)) {
    comm_release(h, true);
    return fail(GF_ECOMM, "fe_sync: a collective did not complete within the timeout (a rank stopped "
                          "responding); communicator aborted, the handle keeps stepping");
  }
  // both streams are idle now: the next step may split at once. main_dirty (set by
  // use_dev) stays: a zero-copy consumer may enqueue reads of the outputs on `stream`
  // after this call, and the next step's second half must wait for them
  h->other_work = false;
  return GF_OK;
}

int fe_set_streams(fe_handle* h, int n) {
  if (!h || (n != 1 && n != 2)) return fail(GF_EINVAL, "n must be 1 or 2");
  if (int rc = use_dev(h)) return rc;
  h->nsplit = n;
  return GF_OK;
}

int fe_join(fe_handle* h) {
  if (!h) return fail(GF_EINVAL, "null handle");
  return use_dev(h);
}

int fe_kernel_timing(fe_handle* h, int enable, double* avg_ms, int64_t* launches) {
  if (!h) return fail(GF_EINVAL, "null handle");
  const bool ow = h->other_work;
  if (int rc = use_dev(h)) return rc;
  // the window's event marks are not work a step waits on: the first step of a window
  // splits like the rest (main_dirty stays set, so stream2 starts after the mark)
  h->other_work = ow;
  if (enable >= 1) {  // start: time every enable-th step launch
    GF_HIP(hipStreamSynchronize(h->stream));
    h->ev_used = 0;
    h->timing = true;
    h->timing_stride = enable;
    h->timing_count = 0;
    // split steps: one window over all of them (both halves run concurrently, so a
    // launch's own duration is not the step's); stream2 starts after the mark
    h->tw_steps = 0;
    GF_HIP(hipEventRecord(h->tw[0], h->stream));
    return GF_OK;
  }
  if (h->tw_steps > 0) {  // split steps: device time of the window per step
    GF_HIP(hipEventRecord(h->tw[1], h->stream));  // after use_dev's join: both halves
    GF_HIP(hipEventSynchronize(h->tw[1]));
    float ms = 0;
    GF_HIP(hipEventElapsedTime(&ms, h->tw[0], h->tw[1]));
    if (avg_ms) *avg_ms = ms / h->tw_steps;
    if (launches) *launches = h->tw_steps;
    if (enable == 0) h->timing = false;
    else {
      h->tw_steps = 0;
      GF_HIP(hipEventRecord(h->tw[0], h->stream));
    }
    return GF_OK;
  }
  GF_HIP(hipStreamSynchronize(h->stream));
  double tot = 0;
  for (size_t k = 0; k + 1 < h->ev_used; k += 2) {
    float ms = 0;
    GF_HIP(hipEventElapsedTime(&ms, h->ev[k], h->ev[k + 1]));
    tot += ms;
  }
  const int64_t n = (int64_t)(h->ev_used / 2);
  if (avg_ms) *avg_ms = n ? tot / n : 0.0;
  if (launches) *launches = n;
  if (enable == 0) h->timing = false;
  return GF_OK;
}

int fe_diag(fe_handle* h, int what, int reps, double* avg_ms) {
  if (!h || reps < 1) return fail(GF_EINVAL, "bad argument");
  if (int rc = use_dev(h)) return rc;
  if (what >= 0x10000) {  // set ablation switches (all bits but 0x10000) for subsequent launches
#ifdef GF_DIAG
    h->diag = what & ~0x10000;
    return GF_OK;
#else
    return fail(GF_EINVAL, "ablation switches need the diagnostic build (make -C gym-flock_amd/csrc diag)");
#endif
  }
  hipEvent_t e0, e1;
  GF_HIP(hipEventCreate(&e0));
  GF_HIP(hipEventCreate(&e1));
  const size_t bytes = h->BN * (size_t)h->cfg.n_agents * 4;
  GF_HIP(hipEventRecord(e0, h->stream));
  for (int r = 0; r < reps; ++r) {
    hipError_t e = gf::launch_fill(h->net, bytes, what == 1, h->stream);
    if (e != hipSuccess) return fail_hip("fill launch", e);
  }
  GF_HIP(hipEventRecord(e1, h->stream));
  GF_HIP(hipEventSynchronize(e1));
  float ms = 0;
  GF_HIP(hipEventElapsedTime(&ms, e0, e1));
  if (avg_ms) *avg_ms = ms / reps;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return GF_OK;
}

// ------------------------------------------------------------------ RCCL metrics path
int fe_comm_unique_id(uint8_t id[128]) {
  if (!id) return fail(GF_EINVAL, "null argument");
  ncclUniqueId uid;
  ncclResult_t r = ncclGetUniqueId(&uid);
  if (r != ncclSuccess) return fail(GF_ECOMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  static_assert(sizeof(uid) == 128, "ncclUniqueId size");
  std::memcpy(id, &uid, 128);
  return GF_OK;
}

int fe_check_shard_sizes(int nranks, const int32_t* n_envs) {
  if (nranks < 1 || !n_envs) return fail(GF_EINVAL, "bad argument");
  for (int r = 0; r < nranks; ++r)
    if (n_envs[r] < 1) {
      std::string m = "bad env shard sizes over ranks (every rank holds at least one env): n_envs =";
      for (int q = 0; q < nranks; ++q) m += " " + std::to_string(n_envs[q]);
      return fail(GF_ECOMM, m);
    }
  return GF_OK;
}

}  // extern "C"

namespace {
// A non-blocking communicator's pending work: poll its async error until it leaves
// ncclInProgress or the deadline passes; then the metrics path is torn down (the
// communicator aborted), so no rank waits forever on a peer that never joined or died.
int comm_wait(fe_handle* h, Clock::time_point deadline, const char* what) {
  for (;;) {
    ncclResult_t st = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(h->comm, &st);
    if (r != ncclSuccess) st = r;
    if (st == ncclSuccess) return GF_OK;
    if (st != ncclInProgress || Clock::now() > deadline) {
      comm_release(h, true);
      h->comm_lost = std::string(what) + ": " +
                     (st != ncclInProgress ? std::string(ncclGetErrorString(st))
                                           : std::string("timed out (a rank did not join or stopped responding)")) +
                     "; communicator aborted";
      return fail(GF_ECOMM, h->comm_lost);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// Wait for side-stream work `seq` on completion word `word` (a gather's staging copy or
// its collective), polling the communicator's async error beside it: on expiry of the
// collective timeout (a rank that died mid-run never posts its part) or a communicator
// error the metrics path is torn down (GF_ECOMM, comm_lost says why); a side stream that
// finished without the word is a HIP error (the path stays up).
int stage_wait(fe_handle* h, int word, uint32_t seq, const char* what) {
  const auto deadline = deadline_in(h->comm_timeout);
  for (int spin = 0;; ++spin) {
    h->dbg[7] = spin;
    if (stage_complete(h, word, seq)) return GF_OK;
    if ((spin & 63) == 63) {
      const hipError_t q = hipStreamQuery(h->comm_stream);
      if (q == hipSuccess && !stage_complete(h, word, seq))
        return fail(GF_EHIP, std::string(what) + ": the side stream finished without the copy's completion word");
      if (q != hipSuccess && q != hipErrorNotReady) return fail_hip(what, q);
    }
    ncclResult_t st = ncclSuccess;
    ncclResult_t r = ncclCommGetAsyncError(h->comm, &st);
    if (r != ncclSuccess) st = r;
    if (spin == 0) h->dbg[3] = static_cast<int32_t>(st);
    const bool err = st != ncclSuccess && st != ncclInProgress;
    if (err || Clock::now() > deadline) {
      comm_release(h, true);
      h->comm_lost = std::string(what) + ": " +
                     (err ? std::string(ncclGetErrorString(st)) : std::string("timed out (a rank stopped responding)")) +
                     "; communicator aborted";
      return fail(GF_ECOMM, h->comm_lost);
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// A collective just enqueued on the non-blocking communicator: wait until it is queued.
int comm_enqueued(fe_handle* h, ncclResult_t r, const char* what) {
  if (r == ncclInProgress) return comm_wait(h, deadline_in(h->comm_timeout), what);
  if (r != ncclSuccess) {
    comm_release(h, true);
    h->comm_lost = std::string(what) + ": " + ncclGetErrorString(r) + "; communicator aborted";
    return fail(GF_ECOMM, h->comm_lost);
  }
  return GF_OK;
}

// A zeroed device buffer of the metrics path (the pad columns of the send blocks are
// never written afterwards).
template <class T>
int comm_alloc(fe_handle* h, T** p, size_t count) {
  if (int rc = dalloc(p, count)) return rc;
  if (*p) GF_HIP(hipMemsetAsync(*p, 0, count * sizeof(T), h->comm_stream));
  return GF_OK;
}

// fe_comm_init once the communicator exists: the side stream, the shard-size exchange
// and the gather buffers. On failure the caller tears everything down.
int comm_setup(fe_handle* h, int nranks, int rank, Clock::time_point deadline) {
  GF_HIP(hipStreamCreateWithFlags(&h->comm_stream, hipStreamNonBlocking));
  if (!h->stage_done) {
    void* p = nullptr;
    GF_HIP(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
    h->stage_done = static_cast<uint32_t*>(p);
    for (int w = 0; w < 4; ++w)  // every earlier sequence number: done
      __atomic_store_n(h->stage_done + w, h->stage_seq[w], __ATOMIC_SEQ_CST);
    void* d = nullptr;
    GF_HIP(hipHostGetDevicePointer(&d, p, 0));
    h->stage_done_dev = static_cast<uint32_t*>(d);
  }
  // every rank's shard size, before any gather pads to the largest
  int32_t* dsz = nullptr;
  if (int rc = dalloc(&dsz, (size_t)nranks)) return rc;
  std::vector<int32_t> sizes(nranks);
  const int32_t mine = h->cfg.n_envs;
  int rc = GF_OK;
  const hipError_t e = hipMemcpyAsync(dsz + rank, &mine, 4, hipMemcpyHostToDevice, h->comm_stream);
  if (e != hipSuccess) rc = fail_hip("shard-size upload", e);
  if (rc == GF_OK) {
    const ncclResult_t r = ncclAllGather(dsz + rank, dsz, 1, ncclInt32, h->comm, h->comm_stream);
    rc = (r == ncclSuccess || r == ncclInProgress) ? comm_wait(h, deadline, "shard-size all-gather")
                                                   : fail(GF_ECOMM, std::string("ncclAllGather: ") + ncclGetErrorString(r));
  }
  if (rc == GF_OK) {
    hipError_t q;
    while ((q = hipStreamQuery(h->comm_stream)) == hipErrorNotReady) {
      if (Clock::now() > deadline) break;
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (q == hipErrorNotReady) {
      rc = fail(GF_ECOMM, "shard-size all-gather: timed out (a rank stopped responding)");
    } else if (q != hipSuccess) {
      rc = fail(GF_EHIP, std::string("shard-size all-gather: ") + hipGetErrorString(q));
    } else if (hipMemcpyAsync(sizes.data(), dsz, 4 * (size_t)nranks, hipMemcpyDeviceToHost, h->comm_stream) !=
                   hipSuccess ||
               hipStreamSynchronize(h->comm_stream) != hipSuccess) {
      rc = fail(GF_EHIP, "shard-size copy");
    } else {
      rc = fe_check_shard_sizes(nranks, sizes.data());
    }
  }
  hipFree(dsz);
  if (rc != GF_OK) return rc;
  h->shard_sizes = sizes;
  h->max_envs = *std::max_element(sizes.begin(), sizes.end());
  const size_t W = h->max_envs;
  for (hipEvent_t* e : {&h->step_ev, &h->step_ev2})
    GF_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  if ((rc = comm_alloc(h, &h->gsend, (size_t)kRewardSlots * W)) ||
      (rc = comm_alloc(h, &h->gather, (size_t)nranks * kRewardSlots * W)) || (rc = comm_alloc(h, &h->ssend, W * 2)) ||
      (rc = comm_alloc(h, &h->stats_gather, (size_t)nranks * W * 2)))
    return rc;
  GF_HIP(hipStreamSynchronize(h->comm_stream));
  h->nranks = nranks;
  h->rank = rank;
  h->gathered_upto = h->steps_written;  // the first gather ships the steps after init
  return GF_OK;
}
}  // namespace

extern "C" {

int fe_comm_init_timeout(fe_handle* h, int nranks, int rank, const uint8_t id[128], double timeout_s) {
  if (!h || !id || nranks < 1 || rank < 0 || rank >= nranks || !(timeout_s > 0)) return fail(GF_EINVAL, "bad argument");
  if (h->comm) return fail(GF_ESTATE, "communicator already initialised");
  if (int rc = use_dev(h)) return rc;
  const auto deadline = deadline_in(timeout_s);
  h->comm_timeout = timeout_s;
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  // RCCL's non-blocking init still connects to the bootstrap root inside the call, which
  // waits for every rank: with a rank missing it never returns. The call therefore runs
  // on a thread of its own, which also waits for the communicator to leave
  // ncclInProgress (RCCL's own init thread works on the creating thread's HIP state:
  // with torch's HIP runtime bound, a creating thread that exited first left a corrupted
  // heap) and then parks for the rest of the process instead of exiting. It hands the
  // communicator over through `state`: 0 running, 1 handed over, 2 abandoned by this call
  // at the deadline (the helper then queues what it created for the communicator
  // worker's abort), so exactly one side owns the communicator. This rank then fails
  // with GF_ECOMM, its handle still usable.
  struct InitJob {
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclInProgress;
    std::atomic<int> state{0};
  };
  auto job = std::make_shared<InitJob>();
  const int dev = h->cfg.device;
  std::thread([job, nranks, uid, rank, dev]() {
    hipSetDevice(dev);
    ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
    config.blocking = 0;
    ncclComm_t c = nullptr;
    ncclResult_t rr = ncclCommInitRankConfig(&c, nranks, uid, rank, &config);
    if (c && (rr == ncclSuccess || rr == ncclInProgress)) {
      for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(c, &st);
        rr = q != ncclSuccess ? q : st;
        if (rr != ncclInProgress || job->state.load(std::memory_order_acquire) == 2) break;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      }
    }
    job->comm = c;
    job->r = rr;
    int running = 0;
    if (!job->state.compare_exchange_strong(running, 1, std::memory_order_acq_rel) && c)
      abort_comm_later(c, dev);  // abandoned: nobody else will release it
    park_thread();
  }).detach();
  while (job->state.load(std::memory_order_acquire) != 1) {
    if (Clock::now() > deadline) {
      int running = 0;
      if (job->state.compare_exchange_strong(running, 2, std::memory_order_acq_rel))
        return fail(GF_ECOMM, "ncclCommInitRankConfig: timed out (a rank did not join); the initialisation is aborted behind");
      break;  // handed over just now
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  h->comm = job->comm;
  h->comm_lost.clear();
  const ncclResult_t r = job->r;
  if (r != ncclSuccess && r != ncclInProgress) {
    comm_release(h, true);
    return fail(GF_ECOMM, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
  }
  if (int rc = comm_wait(h, deadline, "ncclCommInitRankConfig")) return rc;
  if (int rc = comm_setup(h, nranks, rank, deadline)) {
    const std::string msg = g_err;
    comm_release(h, true);  // abort: a peer may still be inside the shard-size collective
    return fail(rc, msg);
  }
  return GF_OK;
}

int fe_comm_init(fe_handle* h, int nranks, int rank, const uint8_t id[128]) {
  return fe_comm_init_timeout(h, nranks, rank, id, kCommInitTimeoutS);
}

int fe_comm_info(fe_handle* h, int32_t* count, int32_t* user_rank, int32_t* device, char* bus_id, int bus_id_len) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->comm) return no_comm(h);
  int c = 0, ur = 0, d = 0;
  ncclResult_t r = ncclCommCount(h->comm, &c);
  if (r == ncclSuccess) r = ncclCommUserRank(h->comm, &ur);
  if (r == ncclSuccess) r = ncclCommCuDevice(h->comm, &d);
  if (r != ncclSuccess) return fail(GF_ECOMM, std::string("ncclComm query: ") + ncclGetErrorString(r));
  if (count) *count = c;
  if (user_rank) *user_rank = ur;
  if (device) *device = d;
  if (bus_id && bus_id_len > 0) GF_HIP(hipDeviceGetPCIBusId(bus_id, bus_id_len, d));
  return GF_OK;
}

int fe_comm_shard_sizes(fe_handle* h, int32_t* sizes, int32_t* max_envs) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->comm) return no_comm(h);
  if (sizes) std::copy(h->shard_sizes.begin(), h->shard_sizes.end(), sizes);
  if (max_envs) *max_envs = h->max_envs;
  return GF_OK;
}

}  // extern "C"

namespace {
// A reward gather's staging copy on the side stream: steps [s0, s0 + count) of the ring
// (wrapping) into the padded send block, then `seq` into the page-locked completion word
// with a system-scope release once every read of the ring has returned.
__global__ __launch_bounds__(256) void ring_stage_kernel(const double* ring, int B, int s0, int count, double* gs,
                                                         int W, uint32_t* done, uint32_t seq) {
  const int n = count * B;
  for (int k = threadIdx.x; k < n; k += 256) {
    const int t = k / B, e = k - t * B;
    gs[(size_t)t * W + e] = ring[(size_t)((s0 + t) % kRewardSlots) * B + e];
  }
  __syncthreads();  // every thread's loads returned (its stores used them)
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// After a collective on the side stream: `seq` into its completion word (the stream's
// earlier work, the collective included, is complete when this runs).
__global__ __launch_bounds__(64) void signal_kernel(uint32_t* done, uint32_t seq) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The stats gather's send block: n doubles from the summaries, then `seq` into the
// completion word once every read of them has returned.
__global__ __launch_bounds__(256) void copy_signal_kernel(const double* src, double* dst, int n, uint32_t* done,
                                                          uint32_t seq) {
  for (int k = threadIdx.x; k < n; k += 256) dst[k] = src[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
}  // namespace

extern "C" {

int fe_allgather_rewards(fe_handle* h) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->comm) return no_comm(h);
  // a step-path call: the gather's stream waits for both step streams' latest work
  // (events only), so back-to-back split steps around it stay split and out of phase
  // (use_dev's join would make the next step a single launch)
  if (int rc = use_dev_step(h)) return rc;
  const int64_t first = h->gathered_upto, count = h->steps_written - first;
  if (count <= 0) return fail(GF_ESTATE, "no step since the last reward all-gather");
  if (count > kRewardSlots) {
    // the ranks step in lockstep, so every rank takes this branch at the same call and
    // none is left inside a collective
    h->gathered_upto = h->steps_written;
    return fail(GF_ESTATE, "the rewards of " + std::to_string(count - kRewardSlots) +
                               " step(s) were overwritten before a gather (gather at least every " +
                               std::to_string(kRewardSlots) + " steps)");
  }
  const size_t B = h->cfg.n_envs, W = h->max_envs;
  // the side stream waits for both step streams' latest work (events only; the step
  // streams never wait for the side stream)
  GF_HIP(hipEventRecord(h->step_ev, h->stream));
  GF_HIP(hipStreamWaitEvent(h->comm_stream, h->step_ev, 0));
  if (h->stream2) {
    GF_HIP(hipEventRecord(h->step_ev2, h->stream2));
    GF_HIP(hipStreamWaitEvent(h->comm_stream, h->step_ev2, 0));
  }
  // the steps' ring slots (two runs when they wrap) into the padded send block, behind
  // the previous collective (which read it) on the same stream
  // and their completion into the page-locked word the ring-slot reuse polls: the copy
  // kernel's own store, not an event query ("a step that did not wait")
  double* gs = h->gsend;
  const int s0 = static_cast<int>(first % kRewardSlots);
  const uint32_t seq = ++h->stage_seq[kWordRing];
  hipLaunchKernelGGL(ring_stage_kernel, dim3(1), dim3(256), 0, h->comm_stream, static_cast<const double*>(h->reward_ring),
                     static_cast<int>(B), s0, static_cast<int>(count), gs, static_cast<int>(W),
                     h->stage_done_dev + kWordRing, seq);
  GF_HIP(hipGetLastError());
  h->ring_reads.push_back({first, seq});
  h->dbg[4] = static_cast<int32_t>(h->ring_reads.size());
  h->dbg[5] = stage_complete(h, kWordRing, seq) ? 1 : 0;
  if (int rc = comm_enqueued(h, ncclAllGather(gs, h->gather, (size_t)count * W, ncclFloat64, h->comm, h->comm_stream),
                             "ncclAllGather (rewards)"))
    return rc;
  hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, h->comm_stream, h->stage_done_dev + kWordRewardGather,
                     ++h->stage_seq[kWordRewardGather]);
  GF_HIP(hipGetLastError());
  h->ag_issued = true;
  h->last_count = static_cast<int>(count);
  h->gathered_upto = h->steps_written;
  return GF_OK;
}

int fe_get_gathered_rewards(fe_handle* h, double* dst) {
  if (!h || !dst) return fail(GF_EINVAL, "null argument");
  if (!h->comm) return no_comm(h);
  if (!h->ag_issued) return fail(GF_ESTATE, "no all-gather issued");
  if (int rc = use_dev(h)) return rc;
  if (int rc = stage_wait(h, kWordRewardGather, h->stage_seq[kWordRewardGather], "reward all-gather")) return rc;
  const size_t n = (size_t)h->nranks * h->last_count * h->max_envs;
  return d2h(h, dst, h->gather, n * 8);  // (on the handle's stream: no use of the null stream)
}

int fe_gathered_steps(fe_handle* h) { return h ? h->last_count : 0; }

int fe_allgather_stats(fe_handle* h) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (!h->comm) return no_comm(h);
  if (!h->has_state) return fail(GF_ESTATE, "state not set");
  // the summaries are taken on the whole current state (both step halves joined); the
  // collective then runs on the side stream, like the reward all-gather
  if (int rc = use_dev(h)) return rc;
  if (int rc = stats_summary_dev(h)) return rc;  // (after the previous stats gather, bounded)
  if (!h->comm) return fail(GF_ECOMM, "metrics path torn down: " + h->comm_lost);
  GF_HIP(hipEventRecord(h->step_ev, h->stream));
  GF_HIP(hipStreamWaitEvent(h->comm_stream, h->step_ev, 0));
  // into the padded send block, on the side stream (after the previous stats gather)
  hipLaunchKernelGGL(copy_signal_kernel, dim3(1), dim3(256), 0, h->comm_stream, static_cast<const double*>(h->stats_sum),
                     h->ssend, h->cfg.n_envs * 2, h->stage_done_dev + kWordStatsCopy, ++h->stage_seq[kWordStatsCopy]);
  GF_HIP(hipGetLastError());
  if (int rc = comm_enqueued(h, ncclAllGather(h->ssend, h->stats_gather, (size_t)h->max_envs * 2, ncclFloat64,
                                              h->comm, h->comm_stream),
                             "ncclAllGather (stats)"))
    return rc;
  hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, h->comm_stream, h->stage_done_dev + kWordStatsGather,
                     ++h->stage_seq[kWordStatsGather]);
  GF_HIP(hipGetLastError());
  h->sg_pending = true;
  return GF_OK;
}

int fe_get_gathered_stats(fe_handle* h, double* dst) {
  if (!h || !dst) return fail(GF_EINVAL, "null argument");
  if (!h->comm) return no_comm(h);
  if (!h->sg_pending) return fail(GF_ESTATE, "no stats all-gather issued");
  if (int rc = use_dev(h)) return rc;
  if (int rc = stage_wait(h, kWordStatsGather, h->stage_seq[kWordStatsGather], "stats all-gather")) return rc;
  return d2h(h, dst, h->stats_gather, (size_t)h->nranks * h->max_envs * 2 * sizeof(double));
}

int fe_comm_destroy(fe_handle* h) {
  if (!h) return fail(GF_EINVAL, "null handle");
  if (int rc = use_dev(h)) return rc;
  comm_release(h, false);
  return GF_OK;
}

}  // extern "C"

namespace {
// fe_debug_comm_gate's kernel: one wave that sleeps until the page-locked flag turns
// non-zero or `ticks` of the device's wall clock pass (always bounded).
// flag[1] = 1 once it runs, flag[2] = 1 (opened) or 2 (timed out) as it ends.
__global__ __launch_bounds__(64) void comm_gate_kernel(unsigned* flag, unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) __hip_atomic_store(flag + 1, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned why = 1u;
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
    if (wall_clock64() - t0 > ticks) {
      why = 2u;
      break;
    }
    __builtin_amdgcn_s_sleep(127);
  }
  if (threadIdx.x == 0) __hip_atomic_store(flag + 2, why, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one process-wide gate flag (fine-grained page-locked memory), never freed: a gate
// kernel abandoned with an aborted side stream may still read it
unsigned* gate_flag() {
  static unsigned* f = [] {
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return (unsigned*)nullptr;
    *static_cast<unsigned*>(p) = 1u;
    return static_cast<unsigned*>(p);
  }();
  return f;
}

// the path of the shared object that defines the function at `fn`
void so_path(const void* fn, char* dst, int len) {
  if (!dst || len <= 0) return;
  Dl_info info{};
  const char* p = (dladdr(fn, &info) && info.dli_fname) ? info.dli_fname : "";
  std::snprintf(dst, (size_t)len, "%s", p);
}
}  // namespace

extern "C" {

int fe_debug_comm_gate(fe_handle* h, int close, double max_seconds) {
  if (!h) return fail(GF_EINVAL, "null handle");
  unsigned* f = gate_flag();
  if (!f) return fail(GF_ENOMEM, "gate flag: hipHostMalloc failed");
  if (!close) {  // also after the communicator was aborted (its side stream abandoned)
    __atomic_store_n(f, 1u, __ATOMIC_SEQ_CST);
    return GF_OK;
  }
  if (!h->comm || !h->comm_stream) return fail(GF_ESTATE, "no communicator (fe_comm_init first)");
  if (!(max_seconds > 0) || max_seconds > 120) return fail(GF_EINVAL, "max_seconds must be in (0, 120]");
  GF_HIP(hipSetDevice(h->cfg.device));
  int khz = 0;
  GF_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->cfg.device));
  void* df = nullptr;
  GF_HIP(hipHostGetDevicePointer(&df, f, 0));
  __atomic_store_n(f + 1, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(f + 2, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(f, 0u, __ATOMIC_SEQ_CST);
  const unsigned long long ticks = static_cast<unsigned long long>(max_seconds * 1000.0 * (khz > 0 ? khz : 100000));
  hipLaunchKernelGGL(comm_gate_kernel, dim3(1), dim3(64), 0, h->comm_stream, static_cast<unsigned*>(df), ticks);
  GF_HIP(hipGetLastError());
  h->dbg[6] = static_cast<int32_t>(hipStreamQuery(h->comm_stream));
  return GF_OK;
}

int fe_debug_comm_state(fe_handle* h, int32_t* out) {
  if (!h || !out) return fail(GF_EINVAL, "null argument");
  for (int k = 0; k < 8; ++k) out[k] = h->dbg[k];
  unsigned* f = gate_flag();
  out[8] = f ? static_cast<int32_t>(__atomic_load_n(f + 1, __ATOMIC_SEQ_CST)) : -1;
  out[9] = f ? static_cast<int32_t>(__atomic_load_n(f + 2, __ATOMIC_SEQ_CST)) : -1;
  out[10] = h->comm ? 1 : 0;
  out[11] = static_cast<int32_t>(h->ring_reads.size());
  return GF_OK;
}

int fe_runtime_info(int32_t* hip_runtime_version, int32_t* hip_driver_version, int32_t* rccl_version, char* hip_path,
                    int hip_path_len, char* rccl_path, int rccl_path_len) {
  int v = 0;
  if (hip_runtime_version) *hip_runtime_version = hipRuntimeGetVersion(&v) == hipSuccess ? v : 0;
  v = 0;
  if (hip_driver_version) {
    *hip_driver_version = hipDriverGetVersion(&v) == hipSuccess ? v : 0;
    (void)hipGetLastError();
  }
  v = 0;
  if (rccl_version) *rccl_version = ncclGetVersion(&v) == ncclSuccess ? v : 0;
  so_path(reinterpret_cast<const void*>(&hipRuntimeGetVersion), hip_path, hip_path_len);
  so_path(reinterpret_cast<const void*>(&ncclGetVersion), rccl_path, rccl_path_len);
  return GF_OK;
}

}  // extern "C"
