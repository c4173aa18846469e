// heat3d-mi355x — command line driver.
//
//   heat3d NX NY NZ ITER_MAX EPS [--flags]
//
// Same positional contract, banner and run report as the reference
// (heat3D.cu:270-315 and 1078-1106; exact formats in SURVEY.md App. B.4).
// Multi-process runs read RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
// MASTER_PORT (torchrun or mpirun env); every rank validates the command line
// (the reference only checked argc on rank 0).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <iostream>
#include <thread>
#include <vector>

#include "../compat/reference_scheme.hpp"
#include "../core/config.hpp"
#include "../core/decomp.hpp"
#include "../comm/comm.hpp"
#include "../io/io.hpp"
#include "../runtime/backend.hpp"
#include "../runtime/solver.hpp"

using namespace heat3d;

// --scheme reference: the reference's own decomposition, emulated in-process
// (SURVEY.md App. B.3b); report lines as the reference printed them.
// Single-step-equivalent HBM traffic (read + write of every point per
// iteration, 2 * sizeof(Real) bytes): comparable with the copy bandwidth;
// temporally blocked sweeps move less, so this can exceed the HBM rate.
static double eff_tbps(double glups, heat3d::DType t) {
  return glups * 2.0 * (double)heat3d::dtype_size(t) / 1e3;
}

static int run_reference_scheme(const Config& cfg) {
  const int P = cfg.virtual_ranks;
  std::array<int, 3> dims = cfg.decomp;
  if (dims[0] * dims[1] * dims[2] == 0) dims = dims_create(P, dims);
  ReferenceScheme rs(cfg.n, dims);
  if (!cfg.quiet) std::cout << cfg.echo_banner() << std::flush;
  ReferenceSchemeResult r = rs.run(cfg.iter_max, cfg.eps, cfg.verbose);
  std::printf("Computational time (parallel): %.6f\n\n", r.seconds);
  if (r.converged)
    std::printf("Simulation has converged in %lld iterations with a convergence threshold of %e\n",
                (long long)r.conv_iter, cfg.eps);
  else
    std::printf("Simulation did not converge within %lld iterations.\n", (long long)cfg.iter_max);
  std::printf("L2-norm error: %.4f %%\n", 100.0 * r.error_rank0);
  std::printf("heat3d: scheme=reference ranks=%d dims=%dx%dx%d chunk=%lldx%lldx%lld norm_rank0=%.6e "
              "global_error=%.4f%%\n",
              rs.ranks(), dims[0], dims[1], dims[2], (long long)rs.chunk()[0], (long long)rs.chunk()[1],
              (long long)rs.chunk()[2], r.norm_rank0, 100.0 * r.error_global);
  std::fflush(stdout);
  std::string out = cfg.output;
  const double pts = (double)cfg.n[0] * cfg.n[1] * cfg.n[2];
  if (out == "auto") out = pts <= 2.2e6 ? "output/out.dat" : "none";
  if (out != "none") rs.write_tecplot(out);
  if (!cfg.json_out.empty()) {
    io::Json j;
    j.set("scheme", std::string("reference"));
    j.set_raw("dims", "[" + std::to_string(dims[0]) + ", " + std::to_string(dims[1]) + ", " +
                          std::to_string(dims[2]) + "]");
    j.set_bool("converged", r.converged);
    j.set("conv_iter", (int64_t)r.conv_iter);
    j.set("iterations", (int64_t)r.iterations);
    j.set("seconds", r.seconds);
    j.set("norm_rank0", r.norm_rank0);
    j.set("error_percent_rank0_local", 100.0 * r.error_rank0);
    j.set("error_percent_global", 100.0 * r.error_global);
    io::write_file_atomic(cfg.json_out, j.dump() + "\n");
  }
  return 0;
}

// One rank's run: banner, time loop, report (heat3D.cu:1078-1106), output.
// Collective calls (run, compute_error, write_tecplot) are made by every rank.
static int drive(const Config& cfg, Solver& solver) {
  const bool root = solver.is_root();
  if (root && !cfg.quiet) std::cout << cfg.echo_banner() << std::flush;
  solver.initialize();
  RunResult r = solver.run();
  double gerr = 0, lerr = 0;
  solver.compute_error(&gerr, &lerr);
  if (root) {
    std::printf("Computational time (parallel): %.6f\n\n", r.seconds);
    if (r.converged)
      std::printf("Simulation has converged in %lld iterations with a convergence threshold of %e\n",
                  (long long)r.conv_iter, cfg.eps);
    else
      std::printf("Simulation did not converge within %lld iterations.\n", (long long)cfg.iter_max);
    std::printf("L2-norm error: %.4f %%\n", 100.0 * (cfg.compat ? lerr : gerr));
    if (!cfg.compat) {
      const auto& d = solver.decomposition();
      std::printf("heat3d: backend=%s comm=%s ranks=%d dims=%dx%dx%d dtype=%s kernel=%s "
                  "iterations=%lld issued=%lld GLUPS=%.3f eff_TBps=%.3f norm=%.6e last_residual=%.6e\n",
                  solver.backend().name(), solver.comm().name(), solver.comm().size(),
                  d.topo.dims[0], d.topo.dims[1], d.topo.dims[2], dtype_name(cfg.dtype),
                  solver.kernel_name().c_str(), (long long)r.iterations, (long long)r.issued,
                  r.glups, eff_tbps(r.glups, cfg.dtype), r.norm, r.last_residual);
    }
    if (cfg.timers) {
      std::printf("heat3d: phase timing (ms/iteration, synchronised):");
      for (auto& pt : solver.phase_times()) std::printf(" %s=%.4f", pt.first.c_str(), pt.second);
      std::printf("\n");
    }
    if (r.fault) std::fprintf(stderr, "heat3d: non-finite residual detected at iteration %lld\n",
                              (long long)r.conv_iter);
    std::fflush(stdout);
  }
  // output/out.dat (heat3D.cu:1109-1179): on by default for small grids
  std::string out = cfg.output;
  const double pts = (double)cfg.n[0] * cfg.n[1] * cfg.n[2];
  if (out == "auto") out = pts <= 2.2e6 ? "output/out.dat" : "none";
  if (out != "none") solver.write_tecplot(out, cfg.tecplot_layout);
  if (!cfg.json_out.empty() && root) {
    io::Json j;
    j.set_raw("N", "[" + std::to_string(cfg.n[0]) + ", " + std::to_string(cfg.n[1]) + ", " +
                       std::to_string(cfg.n[2]) + "]");
    j.set("dtype", std::string(dtype_name(cfg.dtype)));
    j.set("backend", std::string(solver.backend().name()));
    j.set("comm", std::string(solver.comm().name()));
    j.set("ranks", (int64_t)solver.comm().size());
    const auto& d = solver.decomposition();
    j.set_raw("dims", "[" + std::to_string(d.topo.dims[0]) + ", " + std::to_string(d.topo.dims[1]) +
                          ", " + std::to_string(d.topo.dims[2]) + "]");
    j.set("kernel", solver.kernel_name());
    j.set("eps", cfg.eps);
    j.set("iter_max", (int64_t)cfg.iter_max);
    j.set_bool("converged", r.converged);
    j.set("conv_iter", (int64_t)r.conv_iter);
    j.set("iterations", (int64_t)r.iterations);
    j.set("issued", (int64_t)r.issued);
    j.set("seconds", r.seconds);
    j.set("glups", r.glups);
    j.set("effective_tbps", eff_tbps(r.glups, cfg.dtype));
    j.set("norm", r.norm);
    j.set("last_residual", r.last_residual);
    j.set("error_percent", 100.0 * gerr);
    j.set("error_percent_rank0_local", 100.0 * lerr);
    j.set_bool("fault", r.fault);
    j.set("graph_launches", (int64_t)solver.graph_launches());
    j.set("stream_graphs", solver.stream_graphs_state());
    j.set("stream_graphs_canary", solver.stream_graphs_note());
    const HipRuntimeInfo hi = solver.backend().is_gpu() ? hip_runtime_info() : HipRuntimeInfo{};
    j.set("hip_runtime_version", (int64_t)hi.runtime_version);
    j.set("hip_library", hi.library);
    j.set("rccl_version", rccl_version());
    j.set("rccl_library", rccl_library_path());
    io::write_file_atomic(cfg.json_out, j.dump() + "\n");
  }
  return r.fault ? 3 : 0;
}

// --gpus N: one process, N ranks, one host thread per GPU (SURVEY.md L1 /
// M1: the reference's MPI_Init replaced by ncclCommInitAll semantics: one
// ncclUniqueId shared in memory, every thread calls ncclCommInitRank for its
// device).  With --backend cpu the threads talk over loopback TCP sockets.
static int run_threads(const Config& cfg) {
  const int n = cfg.gpus;
  BackendKind bk = cfg.backend;
  if (bk == BackendKind::Auto) bk = hip_device_count() > 0 ? BackendKind::Hip : BackendKind::Cpu;
  std::string uid;
  if (bk == BackendKind::Hip) {
    HEAT3D_CHECK(hip_device_count() >= n, "--gpus " << n << " but " << hip_device_count()
                                                  << " GPU(s) visible (RCCL needs one device per rank)");
    uid = rccl_unique_id();
  }
  const char* bp = std::getenv("HEAT3D_BOOTSTRAP_PORT");
  const int port = bp && *bp ? std::atoi(bp) : 29501;
  std::vector<int> codes(n, 2);
  std::vector<std::thread> threads;
  for (int r = 0; r < n; ++r) {
    threads.emplace_back([&, r] {
      try {
        Config c = cfg;
        c.backend = bk;
        RankPlacement w;
        w.rank = r;
        w.size = n;
        w.local_rank = r;
        w.device = bk == BackendKind::Hip ? r : 0;
        w.bootstrap_port = port;
        w.rccl_uid = uid;
        if (c.comm == CommKind::Auto) c.comm = bk == BackendKind::Hip ? CommKind::Rccl : CommKind::Socket;
        if (bk == BackendKind::Cpu && c.cpu_threads == 0)
          c.cpu_threads = std::max(1, (int)std::thread::hardware_concurrency() / n);
        auto solver = make_solver(c, w);
        codes[r] = drive(c, *solver);
      } catch (const std::exception& e) {
        // a failed rank would leave its peers blocked in collectives: end the job
        std::cerr << "heat3d: rank " << r << " error: " << e.what() << std::endl;
        std::fflush(stdout);
        std::_Exit(2);
      }
    });
  }
  for (auto& t : threads) t.join();
  int code = 0;
  for (int c : codes) code = std::max(code, c);
  return code;
}

int main(int argc, char** argv) {
  Config cfg;
  try {
    cfg = Config::parse(argc, argv);
  } catch (const UsageError& e) {
    // every rank validates (reference heat3D.cu:284-292 checked on rank 0
    // only and let the others run on into stoi); rank 0 prints
    if (rank_from_env() == 0) {
      std::cout << Config::usage() << std::flush;
      std::cerr << "heat3d: " << e.what() << std::endl;
    } else {
      // a launcher (mpirun) tears the job down at the first failed rank: give
      // rank 0's usage text time to be written and forwarded first (without
      // this pause mpirun lost it now and then: tests/test_mpirun_cli.py)
      std::this_thread::sleep_for(std::chrono::milliseconds(500));
    }
    return 1;
  }
  try {
    if (cfg.scheme == "reference") return run_reference_scheme(cfg);
    if (cfg.gpus > 1) return run_threads(cfg);
    auto solver = make_solver_from_env(cfg);
    return drive(cfg, *solver);
  } catch (const std::exception& e) {
    std::cerr << "heat3d: error: " << e.what() << std::endl;
    return 2;
  }
}
