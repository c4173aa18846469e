// heat3d-mi355x — run configuration, physics constants, CLI parsing.
//
// The positional contract `NX NY NZ ITER_MAX EPS` is the reference's
// (heat3D.cu:270-315); physics constants follow heat3D.cu:331-367
// (unit cube, alpha = 1, CFL = 0.4, dt = CFL/6 * min(h)^2, D_d = dt/h_d^2).
// Long flags are new (SURVEY.md §5 "Config / flag system").
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "common.hpp"

namespace heat3d {

struct Physics {
  int64_t n[3] = {0, 0, 0};      // global vertex counts
  double length[3] = {1.0, 1.0, 1.0};
  double alpha = 1.0;
  double cfl = 0.4;
  double h[3] = {0, 0, 0};       // spacing
  double dt = 0;
  double D[3] = {0, 0, 0};       // dt * alpha / h^2 per axis

  static Physics make(int64_t nx, int64_t ny, int64_t nz);
};

enum class BackendKind { Auto, Hip, Cpu };
enum class CommKind { Auto, None, Local, Rccl, Socket };

struct Config {
  // --- reference positional arguments
  int64_t n[3] = {0, 0, 0};
  int64_t iter_max = 0;
  double eps = 0.0;
  std::string eps_text;        // as typed, for the echo banner
  std::string argv0 = "heat3d";

  // --- framework flags
  DType dtype = DType::F64;
  BackendKind backend = BackendKind::Auto;
  CommKind comm = CommKind::Auto;
  std::array<int, 3> decomp = {0, 0, 0};  // 0 = choose with dims_create
  int virtual_ranks = 1;                  // LocalComm: P subdomains in one process
  int gpus = 0;                           // >1: this process runs that many ranks, one host thread per GPU
  int device = -1;                        // -1: LOCAL_RANK or 0
  bool use_graph = true;
  bool overlap = true;
  int check_every = 64;                   // host poll period for the device convergence flag
  int graph_chunk = 0;                    // iterations per captured hipGraph (rounded to even; 0 = auto:
                                          // 32, 96 for the overlapped multi-stream schedule)
  std::string kernel = "auto";            // stencil kernel variant
  std::string kernel2 = "auto";           // 2-step temporally blocked kernel variant
  int temporal = 0;                       // 0 auto (2 on GPU without halos), 1 off, 2 on
  std::string output = "auto";            // path | none | auto (output/out.dat when small)
  std::string tecplot_layout = "auto";    // auto | ref | owned
  bool compat = false;                    // reproduce reference reporting quirks
  // "ghost": this framework's decomposition (default); "reference": emulate
  // the reference's shared-plane scheme (compat/reference_scheme.hpp, CPU)
  std::string scheme = "ghost";
  int64_t checkpoint_every = 0;
  int64_t verify_halo = 0;                // race detection: checksum halos every K iterations
  bool timers = false;                    // per-phase timing (synchronised diagnostic run)
  std::string checkpoint_dir;
  std::string restart;
  std::string json_out;
  int verbose = 0;
  double progress_s = 0;          // run(): stderr heartbeat period (0 = off)
  double time_limit_s = 0;        // run(): wall budget, stop unconverged past it (0 = none)
  // overlapped block sweeps: y / z boundary layers one tile stride thick
  // (whole tiles instead of K-thin ones; --thin-layers: K thick)
  bool tile_layers = true;
  bool quiet = false;
  int cpu_threads = 0;
  int reserve_cus = -1;                   // -1 auto: 8 (one per XCD) for overlapped multi-rank schedules, 0 under long x-slab interiors

  // --- schedule / runtime knobs (until round 2 HEAT3D_* environment variables)
  int lag = -1;                   // lagged convergence check of overlapped sweeps (third buffer): -1 auto, 0 off, 1 on
  bool block_overlap = true;      // block decompositions: interior || halo (false: exchange first)
  // K+1-step sweeps absorb step counts that are not multiples of K: -1 auto
  // (GPU: where timed at start-up cheaper than the partial sweep), 1 always, 0
  // never, 2 timed on any backend (tests of the rank vote on the CPU), 3 as 2
  // and long-major (Solver::long_sweeps_for) whatever the timing
  int long_sweeps = -1;
  // time the interior sweeps' schedule candidates at initialisation: -1 auto
  // (single-subdomain runs, whose sweeps run alone as they are timed), 0 off, 1 on
  int autotune = -1;
  // overlapped multi-stream schedules as hipGraphs too (one linear graph per
  // stream, device-side cross-stream waits): -1 auto (eager: measured faster
  // on the 8-GPU share, Solver::stream_graphs_enabled), 1 on, 0 eager.  Where
  // on, a canary replay at initialisation with a short device-wait timeout
  // (graph_canary_s) decides; a timed-out or pathologically slow replay on any
  // rank turns them off for the job (Solver::canary_stream_graphs).
  int stream_graphs = -1;
  double graph_canary_s = 2.0;    // device-wait timeout of the canary replay (0: no canary)
  // single-subdomain K-step sweeps run their convergence check in the sweep's
  // last workgroup (StencilParams::fuse_check) instead of a kernel after it
  bool fuse_check = true;
  // ... and from each sweep's last residual only (the FTCS residual max-norm
  // is non-increasing; Solver::residual_last_ok, resolve_coarse)
  bool monotone_check = true;
  bool rccl_graph = true;         // RCCL calls may be recorded into hipGraphs (tests/test_gpu_rccl.py)
  bool rccl_shared = false;       // one RCCL communicator for halos and all-reduces (else ncclCommSplit)
  int rccl_p2p_channels = 0;      // RCCL P2P channel pool (NCCL_MAX_P2P_NCHANNELS): N > 0 that many, else RCCL's default
  double mem_reserve_gb = 2.0;    // memory preflight: reserve for RCCL, code objects, scratch
  bool mem_preflight = true;      // refuse configurations that do not fit before allocating
  double host_mem_limit_gb = 0;   // gather-to-root Tecplot: host RAM budget (0 = half of RAM)
  int io_stage_mb = 64;           // output / checkpoint staging chunk
  double watchdog_s = 900;        // abort the communicators after this long without progress
  double fake_allreduce_us = 0;   // diagnostic: emulated all-reduce latency (virtual ranks)
  double phantom_gbps = 50;       // phantom-rank proxy: emulated link rate per peer
  double phantom_allreduce_us = 20;
  int phantom_channels = 4;       // workgroups an emulated transfer holds per peer
  int phantom_allreduce_channels = 2;
  bool phantom_overlap = false;   // --phantom-wire overlap: copies inside the emulated wire time
  bool phantom_paced = false;     // --phantom-wire paced: copies paced at the wire rate for the wire time
  bool phantom_rccl_footprint = false;  // --phantom-footprint rccl|small: stand-in kernels sized as RCCL's

  // Parse argv.  Throws UsageError on a malformed command line.
  static Config parse(int argc, const char* const* argv);
  static std::string usage();
  std::string echo_banner() const;  // the reference's "Runnung ..." block (B.4)
};

class UsageError : public Error {
 public:
  explicit UsageError(const std::string& m) : Error(m) {}
};

std::array<int, 3> parse_decomp(const std::string& s);

}  // namespace heat3d
