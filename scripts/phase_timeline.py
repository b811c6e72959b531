"""Phase timeline of flock_step_kernel at config 2 from a -DGF_STAMPS build
(make -C gym-flock_amd/csrc stamps STAMPS=1|2; GYMFLOCK_LIB=build/lib_stamps1/libgymflock.so).

Per workgroup (lane 0 of wave 0), s_memrealtime stamps (10 ns):
 0 entry  1 rows loaded  2 tile0 published  3 tile0 pass1  4 tile0 features  5 tile1
 published  6 tile1 pass1  7 degrees  8 network stores issued  9 last features  10 end
 11 stores drained (STAMPS=2)  15 HW_ID | XCC_ID << 32
Prints per-phase durations and how many workgroups are in each phase over time."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-flock_amd")]
from gym_flock import _native as nat  # noqa: E402
from gym_flock.init_states import synthetic_batch  # noqa: E402

N, B = int(os.environ.get("N", 1024)), int(os.environ.get("B", 256))  # N=8192 B=16: a config-5 half batch
flags = int(os.environ.get("FLAGS", "0"), 0)
KNN = os.environ.get("KNN") == "1"  # the Flocking-v0 step (fused 7-NN)
h = nat.FlockHandle(N, B, n_neighbors=7 if KNN else 0)
if KNN:
    flags |= nat.FE_WITH_KNN
h.set_streams(1)  # one launch per step: every workgroup of the step has its stamp slots
if os.environ.get("DIAG"):
    h.diag_switches(int(os.environ["DIAG"]))
x0 = synthetic_batch(B, N)
h.set_actions(np.random.RandomState(0).uniform(-1, 1, size=(B, N, 2)).astype(np.float32))
lib = nat.load()
lib.fe_diag_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
G = 8192
bpe = -(-N // (32 if N <= 1024 else 16))
assert B * bpe <= G, "stamp slots cover 8192 workgroups"
buf = np.zeros(G * 16, np.uint64)
runs = []
for rep in range(6):
    h.set_state(x0)
    for _ in range(3):  # back-to-back launches like the bench; stamps are the last one's
        h.step(None, nat.FE_U_RESIDENT | flags)
    h.sync()
    assert lib.fe_diag_stamps(buf.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), G * 16) == 0
    runs.append(buf.reshape(G, 16).copy())

S = runs[-1][:B * bpe]
G = len(S)
t = S[:, :12].astype(np.int64)
t0 = t[:, 0].min()
rel = (t - t0) * 0.01  # us
hw = S[:, 15]
xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xF
hwid = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
cu = (hwid >> 8) & 0xF
sh = (hwid >> 12) & 1
se = (hwid >> 13) & 0x7
cuid = xcc * 1000 + se * 100 + sh * 16 + cu
print("kernel span (first entry -> last end): %.1f us" % (rel[:, 10].max() - rel[:, 0].min()))
if (S[:, 11] > 0).all():
    print("  to last drained: %.1f us" % (rel[:, 11].max()))
print("distinct CUs %d, workgroups per CU: %s" % (len(np.unique(cuid)), np.bincount(np.unique(cuid, return_counts=True)[1])[-8:]))
names = ["rows", "tile0 load", "tile0 pass1", "tile0 feat", "tile1 load", "tile1 pass1", "degree",
         "store issue", "last feat", "epilogue"]
print("%-12s %8s %8s %8s %8s" % ("phase", "median", "p10", "p90", "mean"))
present = [k for k in range(11) if (S[:, k] > 0).all()]  # the split kernel stamps a subset
for k0, k1 in zip(present[:-1], present[1:]):
    d = rel[:, k1] - rel[:, k0]
    nm = names[k1 - 1] if k1 == k0 + 1 else "%d->%d" % (k0, k1)
    print("%-12s %8.2f %8.2f %8.2f %8.2f" % (nm, np.median(d), np.percentile(d, 10), np.percentile(d, 90), d.mean()))
if (S[:, 11] > 0).all():
    d = rel[:, 11] - rel[:, 10]
    print("%-12s %8.2f %8.2f %8.2f %8.2f" % ("drain", np.median(d), np.percentile(d, 10), np.percentile(d, 90), d.mean()))
life = rel[:, 10] - rel[:, 0]
print("lifetime     %8.2f %8.2f %8.2f %8.2f" % (np.median(life), np.percentile(life, 10), np.percentile(life, 90), life.mean()))
# concurrency timeline: workgroups resident, in compute (entry->stores start), storing
# (degree done -> stores issued) and after (stores issued -> end)
span = rel[:, 10].max()
grid = np.arange(0, span, span / 40)
print("%8s %8s %8s %8s %8s" % ("t_us", "resident", "compute", "issuing", "tail"))
for tt in grid:
    res = (rel[:, 0] <= tt) & (rel[:, 10] > tt)
    comp = (rel[:, 0] <= tt) & (rel[:, 7] > tt)
    iss = (rel[:, 7] <= tt) & (rel[:, 8] > tt)
    tail = (rel[:, 8] <= tt) & (rel[:, 10] > tt)
    print("%8.1f %8d %8d %8d %8d" % (tt, res.sum(), comp.sum(), iss.sum(), tail.sum()))
# start times: dispatch order vs time
order = np.argsort(rel[:, 0])
print("entry time of the k-th dispatched workgroup (k=0,1280,2560,...):",
      " ".join("%.1f" % rel[order[k], 0] for k in range(0, G, 1280)))
np.save(os.path.join(ROOT, "gpurun_out", "stamps.npy"), S)
