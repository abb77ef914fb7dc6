// MPI control plane: the reference's own launch model (mpirun / srun, one rank per GPU, the
// control collectives over MPI_COMM_WORLD: src/sequence.cpp:88-125, src/benchmarker.cpp:45-145,
// tenzing-mcts mcts.hpp:149-150).
//
// libmpi is opened at run time, so the build needs no MPI and a process that never asks for the
// MPI backend never loads it. The ABI is MPICH's (MPICH, Cray MPICH, MVAPICH, Intel MPI: handles
// are ints, the constants below are fixed by that ABI); this image ships MPICH 3.3 under
// /opt/conda. MPI is host-only here: it carries the search's small control messages, never
// device buffers (the data plane is RCCL / IPC puts).
#include "ctrl.hpp"
#include "util.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <string>

namespace tz {

namespace {

// MPICH ABI (mpi.h of MPICH 3.x/4.x)
using MPI_Comm = int;
using MPI_Datatype = int;
using MPI_Op = int;
constexpr MPI_Comm kCommWorld = 0x44000000;
constexpr MPI_Datatype kByte = 0x4c00010d;
constexpr MPI_Datatype kInt = 0x4c000405;
constexpr MPI_Datatype kDouble = 0x4c00080b;
constexpr MPI_Op kMax = 0x58000001;
constexpr MPI_Op kSum = 0x58000003;
constexpr int kThreadFunneled = 1;
void *const kInPlace = reinterpret_cast<void *>(-1);

struct Api {
  void *lib = nullptr;
  std::string path;
  int (*Initialized)(int *) = nullptr;
  int (*Finalized)(int *) = nullptr;
  int (*Init_thread)(int *, char ***, int, int *) = nullptr;
  int (*Finalize)() = nullptr;
  int (*Comm_rank)(MPI_Comm, int *) = nullptr;
  int (*Comm_size)(MPI_Comm, int *) = nullptr;
  int (*Barrier)(MPI_Comm) = nullptr;
  int (*Bcast)(void *, int, MPI_Datatype, int, MPI_Comm) = nullptr;
  int (*Allreduce)(const void *, void *, int, MPI_Datatype, MPI_Op, MPI_Comm) = nullptr;
  int (*Allgather)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, MPI_Comm) = nullptr;
  int (*Allgatherv)(const void *, int, MPI_Datatype, void *, const int *, const int *, MPI_Datatype,
                    MPI_Comm) = nullptr;
  int (*Alltoall)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, MPI_Comm) = nullptr;
  int (*Alltoallv)(const void *, const int *, const int *, MPI_Datatype, void *, const int *,
                   const int *, MPI_Datatype, MPI_Comm) = nullptr;
  bool initializedHere = false;
};

template <class F> void sym(Api &a, F &f, const char *name) {
  f = reinterpret_cast<F>(dlsym(a.lib, name));
  TZ_CHECK(f, "MPI library " << a.path << " has no " << name);
}

std::mutex g_mu;
Api *g_api = nullptr; // process-wide: MPI is initialized at most once per process

/// "" if `lib` implements the MPICH ABI (MPICH, Cray MPICH, MVAPICH, Intel MPI), else why not
std::string mpich_abi(void *lib) {
  using GetVersion = int (*)(char *, int *);
  auto get = reinterpret_cast<GetVersion>(dlsym(lib, "MPI_Get_library_version"));
  if (!get) return "no MPI_Get_library_version (not an MPI-3 library)";
  char buf[8192] = {0}; // >= MPI_MAX_LIBRARY_VERSION_STRING of every implementation
  int len = 0;
  if (get(buf, &len) != 0) return "MPI_Get_library_version failed";
  const std::string v(buf, size_t(std::max(0, std::min(len, int(sizeof(buf) - 1)))));
  for (const char *k : {"MPICH", "MVAPICH", "Intel(R) MPI", "CRAY MPICH"})
    if (v.find(k) != std::string::npos) return "";
  return "not an MPICH-ABI library (" + v.substr(0, 60) + ")";
}

void finalize_at_exit() {
  // an MPI launcher counts a rank that exits without MPI_Finalize as failed
  if (g_api && g_api->initializedHere) {
    int fin = 0;
    g_api->Finalized(&fin);
    if (!fin) g_api->Finalize();
  }
}

Api &api(const std::string &want) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api) return *g_api;
  auto *a = new Api();
  std::vector<std::string> tries;
  if (!want.empty()) tries.push_back(want);
  if (const char *e = std::getenv("TZ_MPI_LIB")) tries.push_back(e);
  for (const char *p : {"libmpi.so.12", "libmpi.so", "/opt/conda/lib/libmpi.so.12", "/opt/conda/lib/libmpi.so"})
    tries.push_back(p);
  std::string errs;
  for (const auto &p : tries) {
    // global: MPICH may open its own plugins that resolve against it
    a->lib = dlopen(p.c_str(), RTLD_NOW | RTLD_GLOBAL);
    if (!a->lib) {
      const char *e = dlerror();
      errs += "\n  " + p + ": " + (e ? e : "not found");
      continue;
    }
    // the handle constants above are MPICH's: refuse any other ABI (Open MPI's handles are
    // pointers; passing it these ints would crash). MPI_Get_library_version may be called
    // before MPI_Init (MPI-3).
    const std::string why = mpich_abi(a->lib);
    if (why.empty()) {
      a->path = p;
      break;
    }
    errs += "\n  " + p + ": " + why;
    dlclose(a->lib);
    a->lib = nullptr;
  }
  if (!a->lib) {
    delete a;
    TZ_THROW("MPI control plane: no MPICH-ABI MPI library could be opened (set TZ_MPI_LIB):" << errs);
  }
  sym(*a, a->Initialized, "MPI_Initialized");
  sym(*a, a->Finalized, "MPI_Finalized");
  sym(*a, a->Init_thread, "MPI_Init_thread");
  sym(*a, a->Finalize, "MPI_Finalize");
  sym(*a, a->Comm_rank, "MPI_Comm_rank");
  sym(*a, a->Comm_size, "MPI_Comm_size");
  sym(*a, a->Barrier, "MPI_Barrier");
  sym(*a, a->Bcast, "MPI_Bcast");
  sym(*a, a->Allreduce, "MPI_Allreduce");
  sym(*a, a->Allgather, "MPI_Allgather");
  sym(*a, a->Allgatherv, "MPI_Allgatherv");
  sym(*a, a->Alltoall, "MPI_Alltoall");
  sym(*a, a->Alltoallv, "MPI_Alltoallv");
  int init = 0, fin = 0;
  a->Initialized(&init);
  a->Finalized(&fin);
  TZ_CHECK(!fin, "MPI control plane: MPI was already finalized in this process");
  if (!init) {
    // the search drives MPI from one thread; other threads (watchdog) never call it
    int provided = 0;
    TZ_CHECK(a->Init_thread(nullptr, nullptr, kThreadFunneled, &provided) == 0, "MPI_Init_thread failed");
    a->initializedHere = true;
    std::atexit(finalize_at_exit);
  }
  g_api = a;
  return *a;
}

#define TZ_MPI(call)                                                                               \
  do {                                                                                             \
    const int rc_ = (call);                                                                        \
    TZ_CHECK(rc_ == 0, #call << " failed (MPI error " << rc_ << ")");                              \
  } while (0)

} // namespace

int MpiCtrl::launcher_size() {
  // MPICH hydra / PMI-1 and PMI-2, MVAPICH; Slurm srun (PMIx) exports only the rank through
  // PMIx, so its task count counts only next to a PMI rank. Open MPI's launcher is not an MPICH
  // one: its ranks keep the TCP control plane (tz-search reads OMPI_COMM_WORLD_RANK / _SIZE),
  // even inside a Slurm allocation where Open MPI's ranks also export PMIX_RANK
  if (std::getenv("OMPI_COMM_WORLD_SIZE")) return 1;
  for (const char *v : {"PMI_SIZE", "MV2_COMM_WORLD_SIZE"})
    if (const char *e = std::getenv(v)) return std::atoi(e);
  if (std::getenv("PMIX_RANK") || std::getenv("PMI_RANK"))
    if (const char *e = std::getenv("SLURM_NTASKS")) return std::atoi(e);
  return 1;
}

bool MpiCtrl::launched() {
  // one rank needs no control plane at all: a single process under a PMI environment (a batch
  // system that wraps every job) keeps the plain single-process path
  return launcher_size() > 1;
}

int MpiCtrl::launcher_local_rank() {
  for (const char *v : {"MPI_LOCALRANKID", "MV2_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID",
                        "OMPI_COMM_WORLD_LOCAL_RANK", "PALS_LOCAL_RANKID"})
    if (const char *e = std::getenv(v)) return std::atoi(e);
  return -1;
}

MpiCtrl::MpiCtrl(const std::string &lib) {
  Api &a = api(lib);
  TZ_MPI(a.Comm_rank(kCommWorld, &rank_));
  TZ_MPI(a.Comm_size(kCommWorld, &size_));
  // a library that initialized as a singleton (not the launcher's MPI) makes every process rank
  // 0 of 1: each would run its own search without an error
  if (launched())
    TZ_CHECK(size_ == launcher_size(), "MPI control plane: MPI_COMM_WORLD has " << size_
                                           << " ranks but the launcher started " << launcher_size()
                                           << " (" << a.path << " is not the launcher's MPI?)");
}

std::string MpiCtrl::library() const { return g_api ? g_api->path : ""; }

void MpiCtrl::barrier() { TZ_MPI(g_api->Barrier(kCommWorld)); }

void MpiCtrl::bcast(std::string &data, int root) {
  long long n = rank_ == root ? (long long)data.size() : 0;
  TZ_MPI(g_api->Bcast(&n, int(sizeof(n)), kByte, root, kCommWorld));
  TZ_CHECK(n >= 0 && n < (1ll << 31), "MPI bcast: message of " << n << " bytes");
  if (rank_ != root) data.assign(size_t(n), '\0');
  if (n) TZ_MPI(g_api->Bcast(&data[0], int(n), kByte, root, kCommWorld));
}

void MpiCtrl::allreduce_max(double *v, size_t n) {
  if (n) TZ_MPI(g_api->Allreduce(kInPlace, v, int(n), kDouble, kMax, kCommWorld));
}

void MpiCtrl::allreduce_sum(double *v, size_t n) {
  if (n) TZ_MPI(g_api->Allreduce(kInPlace, v, int(n), kDouble, kSum, kCommWorld));
}

std::vector<std::string> MpiCtrl::allgather(const std::string &mine) {
  TZ_CHECK(mine.size() < (size_t(1) << 31), "MPI allgather: message too large");
  int len = int(mine.size());
  std::vector<int> lens(size_t(size_), 0);
  std::vector<int> offs(size_t(size_), 0);
  TZ_MPI(g_api->Allgather(&len, 1, kInt, lens.data(), 1, kInt, kCommWorld));
  long long total = 0;
  for (int r = 0; r < size_; ++r) {
    offs[size_t(r)] = int(total);
    total += lens[size_t(r)];
  }
  TZ_CHECK(total < (1ll << 31), "MPI allgather: " << total << " bytes in total");
  std::string all(size_t(total), '\0');
  TZ_MPI(g_api->Allgatherv(mine.data(), len, kByte, total ? &all[0] : nullptr, lens.data(), offs.data(),
                           kByte, kCommWorld));
  std::vector<std::string> out(static_cast<size_t>(size_));
  for (int r = 0; r < size_; ++r) out[size_t(r)] = all.substr(size_t(offs[size_t(r)]), size_t(lens[size_t(r)]));
  return out;
}

std::vector<std::string> MpiCtrl::alltoallv(const std::vector<std::string> &out) {
  // each rank moves only its own payloads (the base version's allgather would hand every rank
  // every payload: P x all faces per rank per exchange for the host-staged halo)
  TZ_CHECK(int(out.size()) == size_, "alltoallv: " << out.size() << " payloads for " << size_ << " ranks");
  const size_t P = static_cast<size_t>(size_);
  std::vector<int> sendLen(P, 0), sendOff(P, 0), recvLen(P, 0), recvOff(P, 0);
  long long st = 0;
  for (int r = 0; r < size_; ++r) {
    TZ_CHECK(out[size_t(r)].size() < (size_t(1) << 31), "MPI alltoallv: payload too large");
    sendLen[size_t(r)] = int(out[size_t(r)].size());
    sendOff[size_t(r)] = int(st);
    st += sendLen[size_t(r)];
  }
  TZ_CHECK(st < (1ll << 31), "MPI alltoallv: " << st << " bytes sent in total");
  TZ_MPI(g_api->Alltoall(sendLen.data(), 1, kInt, recvLen.data(), 1, kInt, kCommWorld));
  long long rt = 0;
  for (int r = 0; r < size_; ++r) {
    recvOff[size_t(r)] = int(rt);
    rt += recvLen[size_t(r)];
  }
  TZ_CHECK(rt < (1ll << 31), "MPI alltoallv: " << rt << " bytes received in total");
  std::string sendBuf;
  sendBuf.reserve(size_t(st));
  for (const auto &o : out) sendBuf += o;
  std::string recvBuf(size_t(rt), '\0');
  TZ_MPI(g_api->Alltoallv(st ? sendBuf.data() : nullptr, sendLen.data(), sendOff.data(), kByte,
                          rt ? &recvBuf[0] : nullptr, recvLen.data(), recvOff.data(), kByte,
                          kCommWorld));
  std::vector<std::string> in(static_cast<size_t>(size_));
  for (int r = 0; r < size_; ++r)
    in[size_t(r)] = recvBuf.substr(size_t(recvOff[size_t(r)]), size_t(recvLen[size_t(r)]));
  return in;
}

} // namespace tz
