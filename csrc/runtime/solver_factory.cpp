// heat3d-mi355x — building a Solver for one rank: placement from the
// launcher's environment, backend, communicator (heat3D.cu:203-263).
#include "solver.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <sstream>
#include <thread>

#include <unistd.h>

#include "../comm/net.hpp"
#include "../io/io.hpp"

namespace heat3d {
// ---------------------------------------------------------------------------
static int env_int(const char* a, const char* b, int dflt) {
  const char* v = std::getenv(a);
  if ((!v || !*v) && b) v = std::getenv(b);
  return (v && *v) ? std::atoi(v) : dflt;
}

int rank_from_env() { return env_int("RANK", "OMPI_COMM_WORLD_RANK", env_int("PMI_RANK", nullptr, 0)); }

std::unique_ptr<Solver> make_solver_from_env(const Config& cfg) {
  RankPlacement w;
  w.rank = rank_from_env();
  w.size = env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", env_int("PMI_SIZE", nullptr, 1));
  w.local_rank = env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", env_int("MPI_LOCALRANKID", nullptr, w.rank));
  const char* ma = std::getenv("MASTER_ADDR");
  w.master = ma && *ma ? ma : "127.0.0.1";
  // The native CLI never shares a process with torch, but torchrun's agent owns
  // MASTER_PORT; bootstrap on MASTER_PORT + 1 unless told otherwise.
  w.bootstrap_port = env_int("HEAT3D_BOOTSTRAP_PORT", nullptr, env_int("MASTER_PORT", nullptr, 29500) + 1);
  w.device = cfg.device;
  const char* sp = std::getenv("HEAT3D_SHOW_PLACEMENT");
  if (sp && *sp && sp[0] != '0') {
    // where the launcher's variables put this rank (tests: mpirun / torchrun contracts)
    const char* src = std::getenv("LOCAL_RANK")                   ? "LOCAL_RANK"
                      : std::getenv("OMPI_COMM_WORLD_LOCAL_RANK") ? "OMPI_COMM_WORLD_LOCAL_RANK"
                      : std::getenv("MPI_LOCALRANKID")            ? "MPI_LOCALRANKID"
                                                                  : "rank";
    const int n = cfg.backend == BackendKind::Cpu ? 0 : hip_device_count();
    const int dev = w.device >= 0 ? w.device : (n > 0 ? w.local_rank % n : -1);
    std::fprintf(stderr, "heat3d: placement rank=%d size=%d local_rank=%d from=%s device=%d of %d\n", w.rank, w.size,
                 w.local_rank, src, dev, n);
  }
  return make_solver(cfg, w);
}

std::unique_ptr<Solver> make_solver(const Config& cfg, const RankPlacement& w) {
  const int rank = w.rank, size = w.size, local_rank = w.local_rank;
  const std::string& master = w.master;
  const int bport = w.bootstrap_port;

  BackendKind bk = cfg.backend;
  if (bk == BackendKind::Auto) bk = hip_device_count() > 0 ? BackendKind::Hip : BackendKind::Cpu;
  CommKind ck = cfg.comm;
  if (ck == CommKind::Auto) {
    if (cfg.virtual_ranks > 1) ck = CommKind::Local;
    else if (size > 1) ck = bk == BackendKind::Hip ? CommKind::Rccl : CommKind::Socket;
    else ck = CommKind::None;
  }
  int device = w.device >= 0 ? w.device : 0;
  if (bk == BackendKind::Hip && w.device < 0) {
    const int n = hip_device_count();
    device = n > 0 ? local_rank % n : 0;
  }
  std::unique_ptr<Backend> be = bk == BackendKind::Hip ? make_hip_backend(device) : make_cpu_backend(cfg.cpu_threads);
  std::unique_ptr<Comm> comm;
  int nranks = 1;
  switch (ck) {
    case CommKind::None:
    case CommKind::Auto:
      HEAT3D_CHECK(size == 1, "WORLD_SIZE=" << size << " needs --comm rccl or socket");
      comm = make_local_comm(1);
      nranks = 1;
      break;
    case CommKind::Local:
      HEAT3D_CHECK(size == 1, "--comm local runs in a single process");
      nranks = cfg.virtual_ranks;
      comm = make_local_comm(nranks);
      break;
    case CommKind::Socket: {
      net::Bootstrap boot(rank, size, master, bport);
      comm = make_socket_comm(rank, size, boot);
      if (bk == BackendKind::Hip) comm = make_staged_comm(std::move(comm));
      nranks = size;
      break;
    }
    case CommKind::Rccl: {
      HEAT3D_CHECK(bk == BackendKind::Hip, "RCCL needs the HIP backend");
      if (!w.rccl_uid.empty()) {
        comm = make_rccl_comm(rank, size, w.rccl_uid, device, rccl_options(cfg));
      } else {
        net::Bootstrap boot(rank, size, master, bport);
        std::string uid = rank == 0 ? rccl_unique_id() : std::string();
        auto all = boot.allgather(uid);
        comm = make_rccl_comm(rank, size, all[0], device, rccl_options(cfg));
      }
      nranks = size;
      break;
    }
  }
  std::array<int, 3> fixed = {0, 0, 0};
  if (cfg.decomp[0] > 0) fixed = cfg.decomp;
  std::array<int, 3> dims = dims_create(nranks, fixed);
  return std::unique_ptr<Solver>(new Solver(cfg, std::move(be), std::move(comm), dims));
}

}  // namespace heat3d
