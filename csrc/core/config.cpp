#include "config.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <sstream>

namespace heat3d {

const char* face_name(Face f) {
  static const char* names[] = {"LEFT", "RIGHT", "BOTTOM", "TOP", "BACK", "FRONT"};
  return names[static_cast<int>(f)];
}

const char* dtype_name(DType t) { return t == DType::F64 ? "fp64" : "fp32"; }

DType parse_dtype(const std::string& s) {
  if (s == "fp64" || s == "f64" || s == "double" || s == "float64") return DType::F64;
  if (s == "fp32" || s == "f32" || s == "float" || s == "float32") return DType::F32;
  throw UsageError("unknown dtype '" + s + "' (use fp64 or fp32)");
}

std::string Box::str() const {
  std::ostringstream os;
  os << "[" << lo[0] << "," << hi[0] << ")x[" << lo[1] << "," << hi[1] << ")x[" << lo[2]
     << "," << hi[2] << ")";
  return os.str();
}

Physics Physics::make(int64_t nx, int64_t ny, int64_t nz) {
  Physics p;
  p.n[0] = nx;
  p.n[1] = ny;
  p.n[2] = nz;
  for (int a = 0; a < 3; ++a) {
    HEAT3D_CHECK(p.n[a] >= 3, "grid needs at least 3 vertices per axis, got " << p.n[a]);
    // heat3D.cu:352-355: spacing = L / (N - 1.0)
    p.h[a] = p.length[a] / static_cast<double>(static_cast<double>(p.n[a]) - 1.0);
  }
  const double hmin = std::min({p.h[0], p.h[1], p.h[2]});
  // heat3D.cu:359-360: dt = CFL * 1.0 / (3 * 2) * pow(min(h), 2.0) / alpha
  p.dt = p.cfl * 1.0 / (3 * 2) * std::pow(hmin, 2.0) / p.alpha;
  // heat3D.cu:365-367: D = dt * alpha / pow(h, 2.0)
  for (int a = 0; a < 3; ++a) p.D[a] = p.dt * p.alpha / std::pow(p.h[a], 2.0);
  return p;
}

std::array<int, 3> parse_decomp(const std::string& s) {
  std::array<int, 3> d = {0, 0, 0};
  int idx = 0;
  std::string cur;
  for (char c : s + "x") {
    if (c == 'x' || c == 'X' || c == ',') {
      if (idx >= 3 || cur.empty()) throw UsageError("bad --decomp '" + s + "' (want AxBxC)");
      d[idx++] = std::atoi(cur.c_str());
      cur.clear();
    } else if (c >= '0' && c <= '9') {
      cur += c;
    } else {
      throw UsageError("bad --decomp '" + s + "' (want AxBxC)");
    }
  }
  if (idx != 3 || d[0] < 1 || d[1] < 1 || d[2] < 1)
    throw UsageError("bad --decomp '" + s + "' (want AxBxC, each >= 1)");
  return d;
}

std::string Config::usage() {
  // Text of heat3D.cu:286-290 followed by the framework's flags.
  std::ostringstream os;
  os << "Incorrect number of command line arguments specified, use the following syntax:\n\n"
     << "bin/HeatEquation3D NUM_CELLS_X NUM_CELLS_Y NUM_CELLS_Z ITER_MAX EPS\n"
     << "\nor, using MPI, use the following syntax:\n\n"
     << "mpirun -n NUM_PROCS bin/HeatEquation3D NUM_CELLS_X NUM_CELLS_Y NUM_CELLS_Z ITER_MAX EPS\n"
     << "\nSee source code for additional informations!\n"
     << "\nheat3d (MI355X) options:\n"
     << "  --dtype fp64|fp32         compute precision (default fp64)\n"
     << "  --backend auto|hip|cpu    compute backend (default: hip when a GPU is visible)\n"
     << "  --comm auto|none|local|rccl|socket\n"
     << "                            halo/reduction transport (auto: rccl for multi-process\n"
     << "                            GPU runs, socket for multi-process CPU runs)\n"
     << "  --decomp AxBxC            process grid (default: balanced MPI_Dims_create split)\n"
     << "  --virtual-ranks P         P subdomains in one process (LocalComm)\n"
     << "  --gpus N                  N ranks in this process, one host thread per GPU (RCCL; with\n"
     << "                            --backend cpu: TCP sockets between the threads)\n"
     << "  --device N                GPU ordinal (default LOCAL_RANK)\n"
     << "  --graph / --no-graph      capture iterations in hipGraphs (default on)\n"
     << "  --no-overlap              do not split interior/boundary work\n"
     << "  --check-every K           host poll period of the device convergence flag\n"
     << "  --kernel NAME             single-step kernel (auto|tile[:V:R:WZ:WY:L]|naive)\n"
     << "  --temporal 0|1|K          K-step temporal blocking, K = 2..6 (0 auto: on on the GPU for\n"
     << "                            one subdomain or x slabs; 1 off; results are bitwise identical)\n"
     << "  --kernel2 SPEC            temporally blocked sweep kernel tl2..tl6[:V:R:WZ:WY:L:Q:STORE]\n"
     << "  --output PATH|none        Tecplot output (default output/out.dat for small grids)\n"
     << "  --tecplot-layout auto|ref|owned\n"
     << "  --compat                  reproduce reference reporting quirks\n"
     << "  --scheme ghost|reference  reference: emulate the reference's shared-plane decomposition\n"
     << "                            (edge extrapolation, corner averaging, local norm, any-rank\n"
     << "                            stop; CPU, all ranks of --decomp / --virtual-ranks in-process)\n"
     << "  --checkpoint-every K --checkpoint-dir DIR   periodic binary checkpoints\n"
     << "  --restart DIR             resume from a checkpoint directory\n"
     << "  --json-out PATH           write a JSON run report\n"
     << "  --verify-halo K           race detection: checksum every halo face every K iterations\n"
     << "  --timers                  per-phase GPU timing (synchronised diagnostic run)\n"
     << "  --verbose N               print residual every N iterations\n"
     << "  --progress S              stderr heartbeat (iteration, residual, rate) every S seconds of run()\n"
     << "  --time-limit S            run(): stop (not converged) after about S seconds (0 = no limit)\n"
     << "  --threads N               CPU backend OpenMP threads\n"
     << "  --thin-layers             overlapped block sweeps: K-thick y / z boundary layers (default: one\n"
     << "                            tile stride thick, so that their tiles are not mostly halo)\n"
     << "  --reserve-cus N           CUs kept free of the interior sweep for comm / boundary / check\n"
     << "                            kernels (default: 8 = one per XCD when the overlapped\n"
     << "                            multi-rank schedule runs, else 0)\n"
     << "  --lag auto|on|off         lagged convergence check of overlapped sweeps (3rd field buffer)\n"
     << "  --no-block-overlap        block decompositions: exchange the halo first, then sweep\n"
     << "  --no-long-sweeps          step-count remainders as partial sweeps, not K+1-step sweeps\n"
     << "  --long-sweeps auto|on|off remainders as K+1-step sweeps: auto = where the start-up timing of\n"
     << "                            the sweeps finds them cheaper than a partial sweep (default auto;\n"
     << "                            GPU only, measure = on any backend; major = step counts as\n"
     << "                            K+1-step sweeps wherever they fit, as auto does where they are\n"
     << "                            cheaper per step)\n"
     << "  --autotune auto|on|off    time the sweep schedule candidates (z stride, x segments) at start-up;\n"
     << "                            auto: single-subdomain runs (--no-autotune = off)\n"
     << "  --stream-graphs auto|on|off  the overlapped multi-stream schedule as one linear hipGraph per\n"
     << "                            stream with device-side cross-stream waits, verified at start-up\n"
     << "                            (auto = off: eager measured faster on the 8-GPU share; on = graphs;\n"
     << "                            --no-stream-graphs = off)\n"
     << "  --graph-canary S          device-wait timeout of the start-up canary replay of those graphs; a\n"
     << "                            rank whose replay times out or runs > 2x eager turns them off for the\n"
     << "                            job (default 2; 0 = no canary)\n"
     << "  --no-fused-check          single-subdomain sweeps: a check kernel after each sweep instead of\n"
     << "                            the check in the sweep's last workgroup\n"
     << "  --no-monotone-check       fused checks: every step's residual, not only each sweep's last one\n"
     << "                            (the residual max-norm of FTCS never grows, so the last one decides;\n"
     << "                            the converging sweep is replayed with all residuals for the iteration)\n"
     << "  --no-rccl-graph           never record RCCL calls into hipGraphs (eager multi-rank steps)\n"
     << "  --rccl-shared             one RCCL communicator for halos and all-reduces\n"
     << "  --rccl-p2p-channels N     RCCL P2P channel pool (NCCL_MAX_P2P_NCHANNELS unless set in the\n"
     << "                            environment): N > 0 that many; default RCCL's own (8 on the 2-rank\n"
     << "                            one-GPU rehearsal under RCCL 2.27 drove host memory past 270 GB)\n"
     << "  --mem-reserve-gb G        memory preflight reserve (default 2)\n"
     << "  --no-mem-preflight        skip the memory preflight\n"
     << "  --host-mem-limit-gb G     host RAM budget of the gather-to-root Tecplot (default RAM/2)\n"
     << "  --io-stage-mb M           output / checkpoint staging chunk (default 64)\n"
     << "  --watchdog S              abort after S seconds without progress (default 900)\n"
     << "  --fake-allreduce-us U     diagnostic: emulated all-reduce latency for virtual ranks\n"
     << "  --phantom-gbps G --phantom-allreduce-us U --phantom-channels C --phantom-allreduce-channels C\n"
     << "                            phantom-rank proxy (tools/rank_proxy.py) link emulation\n"
     << "  --phantom-wire serial|overlap|paced  phantom exchange: wire time then copies, copies inside it,\n"
     << "                            or copies paced at the wire rate over the wire time\n"
     << "  --phantom-footprint rccl|small  phantom comm kernels in RCCL's kernel footprint (256 threads,\n"
     << "                            140 VGPRs, 20 KB LDS) or small (64 threads; default)\n"
     << "  --quiet                   suppress the banner\n";
  return os.str();
}

static int64_t to_i64(const std::string& s, const char* what) {
  try {
    size_t pos = 0;
    long long v = std::stoll(s, &pos);
    if (pos != s.size()) throw std::invalid_argument(s);
    return v;
  } catch (const std::exception&) {
    throw UsageError(std::string("invalid integer for ") + what + ": '" + s + "'");
  }
}

static double to_f64(const std::string& s, const char* what) {
  try {
    size_t pos = 0;
    double v = std::stod(s, &pos);
    if (pos != s.size()) throw std::invalid_argument(s);
    return v;
  } catch (const std::exception&) {
    throw UsageError(std::string("invalid number for ") + what + ": '" + s + "'");
  }
}

Config Config::parse(int argc, const char* const* argv) {
  Config c;
  if (argc > 0 && argv[0]) c.argv0 = argv[0];
  std::vector<std::string> pos;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto need = [&](const char* flag) -> std::string {
      if (i + 1 >= argc) throw UsageError(std::string("missing value for ") + flag);
      return argv[++i];
    };
    // accept --flag=value too
    std::string val;
    auto eq = a.find('=');
    bool has_eq = a.rfind("--", 0) == 0 && eq != std::string::npos;
    std::string key = has_eq ? a.substr(0, eq) : a;
    auto get = [&](const char* flag) { return has_eq ? a.substr(eq + 1) : need(flag); };
    if (key.rfind("--", 0) != 0) {
      pos.push_back(a);
      continue;
    }
    if (key == "--dtype") c.dtype = parse_dtype(get("--dtype"));
    else if (key == "--backend") {
      std::string v = get("--backend");
      if (v == "auto") c.backend = BackendKind::Auto;
      else if (v == "hip" || v == "gpu") c.backend = BackendKind::Hip;
      else if (v == "cpu") c.backend = BackendKind::Cpu;
      else throw UsageError("unknown backend '" + v + "'");
    } else if (key == "--comm") {
      std::string v = get("--comm");
      if (v == "auto") c.comm = CommKind::Auto;
      else if (v == "none") c.comm = CommKind::None;
      else if (v == "local") c.comm = CommKind::Local;
      else if (v == "rccl" || v == "nccl") c.comm = CommKind::Rccl;
      else if (v == "socket" || v == "tcp") c.comm = CommKind::Socket;
      else throw UsageError("unknown comm '" + v + "'");
    } else if (key == "--decomp") c.decomp = parse_decomp(get("--decomp"));
    else if (key == "--virtual-ranks") c.virtual_ranks = (int)to_i64(get("--virtual-ranks"), "--virtual-ranks");
    else if (key == "--gpus") c.gpus = (int)to_i64(get("--gpus"), "--gpus");
    else if (key == "--device") c.device = (int)to_i64(get("--device"), "--device");
    else if (key == "--graph") c.use_graph = true;
    else if (key == "--no-graph") c.use_graph = false;
    else if (key == "--overlap") c.overlap = true;
    else if (key == "--no-overlap") c.overlap = false;
    else if (key == "--check-every") c.check_every = (int)to_i64(get("--check-every"), "--check-every");
    else if (key == "--graph-chunk") c.graph_chunk = (int)to_i64(get("--graph-chunk"), "--graph-chunk");
    else if (key == "--kernel") c.kernel = get("--kernel");
    else if (key == "--kernel2") c.kernel2 = get("--kernel2");
    else if (key == "--temporal") {
      c.temporal = (int)to_i64(get("--temporal"), "--temporal");
      if (c.temporal < 0 || c.temporal > 6) throw UsageError("--temporal must be 0 (auto), 1 (off) or 2..6");
    }
    else if (key == "--output") c.output = get("--output");
    else if (key == "--tecplot-layout") c.tecplot_layout = get("--tecplot-layout");
    else if (key == "--compat") c.compat = true;
    else if (key == "--scheme") {
      c.scheme = get("--scheme");
      if (c.scheme != "ghost" && c.scheme != "reference")
        throw UsageError("--scheme must be ghost or reference");
    }
    else if (key == "--checkpoint-every") c.checkpoint_every = to_i64(get("--checkpoint-every"), "--checkpoint-every");
    else if (key == "--verify-halo") c.verify_halo = to_i64(get("--verify-halo"), "--verify-halo");
    else if (key == "--timers") c.timers = true;
    else if (key == "--checkpoint-dir") c.checkpoint_dir = get("--checkpoint-dir");
    else if (key == "--restart") c.restart = get("--restart");
    else if (key == "--json-out") c.json_out = get("--json-out");
    else if (key == "--verbose") c.verbose = (int)to_i64(get("--verbose"), "--verbose");
    else if (key == "--progress") c.progress_s = to_f64(get("--progress"), "--progress");
    else if (key == "--time-limit") c.time_limit_s = to_f64(get("--time-limit"), "--time-limit");
    else if (key == "--threads") c.cpu_threads = (int)to_i64(get("--threads"), "--threads");
    else if (key == "--reserve-cus") c.reserve_cus = (int)to_i64(get("--reserve-cus"), "--reserve-cus");
    else if (key == "--quiet") c.quiet = true;
    else if (key == "--lag") {
      const std::string v = get("--lag");
      if (v == "auto") c.lag = -1;
      else if (v == "on" || v == "1") c.lag = 1;
      else if (v == "off" || v == "0") c.lag = 0;
      else throw UsageError("--lag must be auto, on or off");
    }
    else if (key == "--no-block-overlap") c.block_overlap = false;
    else if (key == "--no-long-sweeps") c.long_sweeps = 0;
    else if (key == "--core-rim" || key == "--no-core-rim" || key == "--halo-chunks")
      throw UsageError(key + " was retired in round 5 (measured slower on every configuration, "
                             "profiles/rank_proxy_r04.md)");
    else if (key == "--thin-layers") c.tile_layers = false;
    else if (key == "--boundary-stream")
      throw UsageError("--boundary-stream was retired in round 5 (the boundary pieces run beside the interior "
                       "on the comm stream; after it was slower on every configuration, profiles/r05/proxy_runs.md)");
    else if (key == "--long-sweeps") {
      const std::string v = get("--long-sweeps");
      if (v == "auto") c.long_sweeps = -1;
      else if (v == "on") c.long_sweeps = 1;
      else if (v == "off") c.long_sweeps = 0;
      else if (v == "measure") c.long_sweeps = 2;  // time the sweeps on any backend (tests)
      else if (v == "major") c.long_sweeps = 3;    // measure, and run long-major whatever the timing
      else throw UsageError("--long-sweeps takes auto, on, off, measure or major");
    }
    else if (key == "--no-autotune") c.autotune = 0;
    else if (key == "--autotune") {
      const std::string v = get("--autotune");
      if (v == "auto") c.autotune = -1;
      else if (v == "on") c.autotune = 1;
      else if (v == "off") c.autotune = 0;
      else throw UsageError("--autotune auto|on|off, not '" + v + "'");
    }
    else if (key == "--no-stream-graphs") c.stream_graphs = 0;
    else if (key == "--stream-graphs") {
      const std::string v = get("--stream-graphs");
      if (v != "auto" && v != "on" && v != "off") throw UsageError("--stream-graphs auto|on|off");
      c.stream_graphs = v == "auto" ? -1 : v == "on" ? 1 : 0;
    }
    else if (key == "--graph-canary") c.graph_canary_s = to_f64(get("--graph-canary"), "--graph-canary");
    else if (key == "--no-fused-check") c.fuse_check = false;
    else if (key == "--no-monotone-check") c.monotone_check = false;
    else if (key == "--rccl-graph") c.rccl_graph = true;
    else if (key == "--no-rccl-graph") c.rccl_graph = false;
    else if (key == "--rccl-shared") c.rccl_shared = true;
    else if (key == "--rccl-p2p-channels") c.rccl_p2p_channels = (int)to_i64(get("--rccl-p2p-channels"), "--rccl-p2p-channels");
    else if (key == "--mem-reserve-gb") c.mem_reserve_gb = to_f64(get("--mem-reserve-gb"), "--mem-reserve-gb");
    else if (key == "--no-mem-preflight") c.mem_preflight = false;
    else if (key == "--host-mem-limit-gb") c.host_mem_limit_gb = to_f64(get("--host-mem-limit-gb"), "--host-mem-limit-gb");
    else if (key == "--io-stage-mb") c.io_stage_mb = (int)to_i64(get("--io-stage-mb"), "--io-stage-mb");
    else if (key == "--watchdog") c.watchdog_s = to_f64(get("--watchdog"), "--watchdog");
    else if (key == "--fake-allreduce-us") c.fake_allreduce_us = to_f64(get("--fake-allreduce-us"), "--fake-allreduce-us");
    else if (key == "--phantom-gbps") c.phantom_gbps = to_f64(get("--phantom-gbps"), "--phantom-gbps");
    else if (key == "--phantom-wire") {
      const std::string v = get("--phantom-wire");
      if (v != "serial" && v != "overlap" && v != "paced") throw UsageError("--phantom-wire serial|overlap|paced");
      c.phantom_overlap = v == "overlap";
      c.phantom_paced = v == "paced";
    }
    else if (key == "--phantom-footprint") {
      const std::string v = get("--phantom-footprint");
      if (v != "rccl" && v != "small") throw UsageError("--phantom-footprint rccl|small");
      c.phantom_rccl_footprint = v == "rccl";
    }
    else if (key == "--phantom-allreduce-us")
      c.phantom_allreduce_us = to_f64(get("--phantom-allreduce-us"), "--phantom-allreduce-us");
    else if (key == "--phantom-channels") c.phantom_channels = (int)to_i64(get("--phantom-channels"), "--phantom-channels");
    else if (key == "--phantom-allreduce-channels")
      c.phantom_allreduce_channels = (int)to_i64(get("--phantom-allreduce-channels"), "--phantom-allreduce-channels");
    else if (key == "--help") throw UsageError("help requested");
    else throw UsageError("unknown option '" + a + "'");
  }
  if (pos.size() != 5)
    throw UsageError("expected 5 positional arguments (NX NY NZ ITER_MAX EPS), got " +
                     std::to_string(pos.size()));
  c.n[0] = to_i64(pos[0], "NUM_CELLS_X");
  c.n[1] = to_i64(pos[1], "NUM_CELLS_Y");
  c.n[2] = to_i64(pos[2], "NUM_CELLS_Z");
  c.iter_max = to_i64(pos[3], "ITER_MAX");
  c.eps = to_f64(pos[4], "EPS");
  c.eps_text = pos[4];
  for (int a = 0; a < 3; ++a)
    if (c.n[a] < 3) throw UsageError("each grid extent must be >= 3");
  if (c.iter_max < 0) throw UsageError("ITER_MAX must be >= 0");
  if (c.virtual_ranks < 1) throw UsageError("--virtual-ranks must be >= 1");
  if (c.gpus < 0) throw UsageError("--gpus must be >= 1");
  if (c.gpus > 1 && c.virtual_ranks > 1) throw UsageError("--gpus and --virtual-ranks are exclusive");
  if (c.check_every < 1) c.check_every = 1;
  if (c.graph_chunk < 0) c.graph_chunk = 0;
  if (c.graph_chunk == 1) c.graph_chunk = 2;
  if (c.graph_chunk % 2) c.graph_chunk += 1;
  if (c.io_stage_mb < 1) c.io_stage_mb = 1;
  if (c.watchdog_s <= 0) throw UsageError("--watchdog must be > 0");
  if (c.progress_s < 0) throw UsageError("--progress must be >= 0");
  if (c.time_limit_s < 0) throw UsageError("--time-limit must be >= 0");
  return c;
}

std::string Config::echo_banner() const {
  // heat3D.cu:293-302 (including the "Runnung" typo and trailing space, B.4).
  std::ostringstream os;
  os << "Runnung HeatEquation3D with the following arguments: \n";
  os << "executable:               " << argv0 << "\n";
  os << "number of cells in x:     " << n[0] << "\n";
  os << "number of cells in y:     " << n[1] << "\n";
  os << "number of cells in z:     " << n[2] << "\n";
  os << "max number of iterations: " << iter_max << "\n";
  os << "convergence threshold:    " << eps << "\n\n";
  return os.str();
}

}  // namespace heat3d
