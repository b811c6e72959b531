// Where does a lone rank of a 2-rank non-blocking RCCL communicator spend its time?
// Each stage prints its elapsed time (stderr, unbuffered). hipcc -o build/comm_probe
// scripts/comm_probe.cpp -lrccl
#include <rccl/rccl.h>
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <thread>

static double now() {
  using namespace std::chrono;
  static const auto t0 = steady_clock::now();
  return duration<double>(steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;  // 0: abort inline, 1: abort on a detached thread, 2: no abort
  hipSetDevice(0);
  ncclUniqueId id;
  fprintf(stderr, "%.3f getUniqueId -> %d\n", now(), (int)ncclGetUniqueId(&id));
  ncclComm_t comm = nullptr;
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclResult_t r = ncclCommInitRankConfig(&comm, 2, id, 0, &cfg);
  fprintf(stderr, "%.3f initRankConfig -> %d comm=%p\n", now(), (int)r, (void*)comm);
  ncclResult_t st = ncclInProgress;
  const double t1 = now();
  while (now() - t1 < 5.0) {
    ncclResult_t q = ncclCommGetAsyncError(comm, &st);
    if (q != ncclSuccess || st != ncclInProgress) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  fprintf(stderr, "%.3f after polling: state %d\n", now(), (int)st);
  if (mode == 0) {
    ncclResult_t a = ncclCommAbort(comm);
    fprintf(stderr, "%.3f abort -> %d\n", now(), (int)a);
  } else if (mode == 1) {
    std::thread([comm] { ncclCommAbort(comm); }).detach();
    fprintf(stderr, "%.3f abort handed to a detached thread\n", now());
  }
  // the device still works
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, 1 << 20);
  e = hipMemset(p, 1, 1 << 20);
  e = hipDeviceSynchronize();
  fprintf(stderr, "%.3f device ok: %s\n", now(), hipGetErrorString(e));
  hipFree(p);
  fprintf(stderr, "%.3f exiting\n", now());
  return 0;
}
