#include "solver.hpp"

#include <algorithm>
#include <atomic>
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

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include "../comm/net.hpp"
#include "../io/io.hpp"

namespace heat3d {

// HEAT3D_SEGV_TRACE=1: (re-)install a fatal-signal handler printing the
// native backtrace right before a graph capture (the HIP / torch runtimes
// install their own handlers after the Python extension's).
static void segv_trace_handler(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "\nheat3d: fatal signal, native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
static void arm_segv_trace() {
  const char* e = std::getenv("HEAT3D_SEGV_TRACE");
  if (!e || !*e || e[0] == '0') return;
  // an alternate signal stack, so that a stack overflow is reported too
  static char* alt = nullptr;
  if (!alt) {
    alt = new char[1 << 16];
    stack_t ss{};
    ss.ss_sp = alt;
    ss.ss_size = 1 << 16;
    sigaltstack(&ss, nullptr);
  }
  struct sigaction sa {};
  sa.sa_handler = segv_trace_handler;
  sa.sa_flags = SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  for (int s : {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT}) sigaction(s, &sa, nullptr);
}

// ---------------------------------------------------------------------------
// KernelSpec
KernelSpec KernelSpec::parse(const std::string& s) {
  KernelSpec k;
  if (s.empty() || s == "auto") return k;
  std::vector<std::string> parts;
  std::stringstream ss(s);
  std::string p;
  while (std::getline(ss, p, ':')) parts.push_back(p);
  const std::string& h = parts[0];
  if (h == "naive") {
    k.kind = Naive;
  } else if (h == "tile" || (h.size() == 3 && h[0] == 't' && h[1] == 'l' && h[2] >= '2' && h[2] <= '6')) {
    // tile = single step; tl2..tl6 = K-step lean sweep kernel
    k.kind = h == "tile" ? Tile : TBL;
    if (k.kind != Tile) k.K = h[2] - '0';
    auto at = [&](std::size_t i) { return parts.size() > i ? std::atoi(parts[i].c_str()) : 0; };
    k.V = at(1);
    k.R = at(2);
    k.WZ = at(3);
    k.WY = at(4);
    k.L = at(5);
    k.NT = at(6);
    if (k.kind != Tile && parts.size() > 7) k.O = at(7);  // store cache-policy bits
    if (k.kind != Tile && parts.size() > 8) k.ZS = at(8);  // z tile stride
  } else if (h == "column" || h == "tb2" || h == "tbk2" || (h.size() == 3 && h[0] == 't' && (h[1] == 'b' || h[1] == 'r'))) {
    throw UsageError("kernel '" + s + "' was retired in round 3 (the column / queue / register-ring kernels); "
                     "use tile for single steps and tl2..tl6 for K-step sweeps");
  } else {
    throw UsageError("unknown kernel '" + s + "' (auto | naive | tile[:V[:R[:WZ[:WY]]]] | "
                     "tl2..tl6[:V[:R[:WZ[:WY[:L[:Q[:STORE[:ZS]]]]]]]])");
  }
  return k;
}

// interior points of an x-slab share above which the overlapped schedule
// runs on every CU (no comm reservation; Solver::Solver): the 2-GPU 1024^3
// share has 5.3e8, the 4-GPU one 2.6e8, the 8-GPU one 1.3e8
constexpr int64_t kLongSlabInterior = 200000000;

KernelSpec KernelSpec::resolved(DType t) const {
  KernelSpec r = *this;
  const bool f64 = t == DType::F64;
  auto def = [](int& f, int v) {
    if (f == 0) f = v;
  };
  switch (kind) {
    case Tile:  // 8-wave tiles, 16 rows x 512 points
      def(r.V, f64 ? 2 : 4);
      def(r.R, 8);
      def(r.WZ, f64 ? 4 : 2);
      def(r.WY, 2);
      break;
    case TBL:  // lean kernel: 16 waves of 64 columns.  fp64: 3 rows per wave
               // (48-row tiles), 2 from K = 4 (32-row tiles: 115 VGPRs, no
               // spill); fp32: 4 rows from K = 4 (64-row tiles)
      // fp32 up to K = 4: packed pairs (V = 2, stencil_tbp.hip: fp64's register
      // shape, 1024^3 tl3:2:3 1450 vs tl4:1:4 1288 GLUPS on one box)
      def(r.V, f64 || K > 4 ? 1 : 2);
      // fp64 K = 4 (the long sweeps of step counts that are not multiples of
      // 3): 12 waves of 3 rows, 144 VGPRs, 750 vs 719 GLUPS for 16 x 2 rows
      // with nt stores on one box
      if (f64 && K == 4 && r.V == 1 && r.R == 0 && r.WY == 0) {
        r.R = 3;
        r.WY = 12;
      }
      // fp64 K = 2 (partial sweeps of multi-rank step-count remainders): 16
      // waves of 5 rows (80-row tiles, 114 VGPRs), nt stores.  Fewer y-halo
      // rows per stored one than 48-row tiles: +7-11% at kernel level on the
      // 1022^3, 508 / 250 / 122-plane slab boxes (profiles/probes_r04.md)
      if (f64 && K == 2 && r.V == 1 && r.R == 0 && r.WY == 0) {
        r.R = 5;
        r.WY = 16;
      }
      // fp64 K = 5 / 6 and fp32 K = 6: no 16-wave shape fits 128 VGPRs
      // without spilling; 8 waves of 3 rows (24-row tiles, up to 256 VGPRs)
      if ((f64 ? K >= 5 : K >= 6) && r.V == 1 && r.R == 0 && r.WY == 0) {
        r.R = 3;
        r.WY = 8;
      }
      // fp64 pairs (V = 2, stencil_tbp.hip): 8 waves (<= 256 VGPRs) of 4 rows,
      // 32 x 128 tiles (K = 2: 6 rows, K = 4: 3 rows)
      if (f64 && r.V == 2 && r.R == 0 && r.WY == 0 && K <= 4) {
        r.R = K == 2 ? 6 : K == 4 ? 3 : 4;
        r.WY = 8;
      }
      def(r.R, (f64 || r.V == 2) ? (K >= 4 ? 2 : 3) : (K == 4 ? 4 : 3));
      def(r.WZ, 1);
      def(r.WY, 16);
      def(r.NT, 3);
      // fp64 default shape: non-temporal output stores (the sweep's output is
      // not re-read before the next sweep; streaming it past L2 keeps the
      // input halo lines resident).  MI355X, 1024^3 kernel level: 756 -> 798
      // GLUPS, 512^3 / 768^3 +2-2.5%
      // (also K = 4, the long sweeps of step counts that are not multiples of
      // 3: 5.45 -> 5.38 ms per 1024^3 sweep.  Not K = 2, the partial sweeps
      // of multi-rank remainders: alone, back to back, nt is faster (1022^3
      // 557 -> 615 GLUPS), but where the solver runs it both policies take
      // 5.3-5.6 ms; profiles/probes_r03.md)
      // fp32 packed-pair default shape too: 1388 -> 1431 GLUPS at 1024^3, 1354
      // -> 1513 at 2049^3
      if (!f64 && r.O < 0 && r.V == 2 && K == 3 && r.R == 3 && r.WY == 16 && r.NT == 3) r.O = 2;
      if (f64 && r.O < 0 && r.V == 2 && r.NT == 3) r.O = 2;
      if (f64 && r.O < 0 && r.V == 1 && r.NT == 3 &&
          ((K == 3 && r.R == 3 && r.WY == 16) || (K == 4 && r.R == 2 && r.WY == 16) ||
           (K == 4 && r.R == 3 && r.WY == 12) || (K == 2 && r.R == 5 && r.WY == 16)))
        r.O = 2;
      break;
    default:
      break;
  }
  return r;
}

std::string KernelSpec::str() const {
  if (kind == Naive) return "naive";
  std::ostringstream os;
  os << (kind == Tile ? std::string("tile:") : "tl" + std::to_string(K) + ":") << V << ":" << R << ":" << WZ << ":"
     << WY << ":" << L << ":" << NT;
  if (kind != Tile && (O > 0 || ZS > 0)) os << ":" << O;
  if (kind != Tile && ZS > 0) os << ":" << ZS;
  return os.str();
}

// ---------------------------------------------------------------------------
static bool trace_on() {
  static const bool on = [] {
    const char* e = std::getenv("HEAT3D_TRACE");
    return e && *e && e[0] != '0';
  }();
  return on;
}
#define H3D_TRACE(msg)                                                   \
  do {                                                                   \
    if (trace_on()) {                                                    \
      std::ostringstream _os;                                            \
      _os << "[heat3d trace] " << msg << "\n";                           \
      std::fputs(_os.str().c_str(), stderr);                             \
      std::fflush(stderr);                                               \
    }                                                                    \
  } while (0)

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

Solver::Solver(const Config& cfg, std::unique_ptr<Backend> be, std::unique_ptr<Comm> comm,
               std::array<int, 3> dims)
    : cfg_(cfg), be_(std::move(be)), comm_(std::move(comm)) {
  dt_ = cfg_.dtype;
  esize_ = dtype_size(dt_);
  phys_ = Physics::make(cfg_.n[0], cfg_.n[1], cfg_.n[2]);
  HEAT3D_CHECK(dims[0] * dims[1] * dims[2] == comm_->size(),
               "process grid " << dims[0] << "x" << dims[1] << "x" << dims[2] << " does not match "
                               << comm_->size() << " ranks");
  dec_ = Decomposition::make(cfg_.n, dims);
  kspec_ = KernelSpec::parse(cfg_.kernel);
  if (kspec_.kind == KernelSpec::TBL) kspec_.kind = KernelSpec::Tile;
  kspec2_ = KernelSpec::parse(cfg_.kernel2);
  overlap_ = cfg_.overlap;

  // K-step temporal blocking: on by default on the GPU, opt-in on the CPU
  // backend (tests).  Depth K from --temporal K, else from --kernel2 tlK,
  // else kDefaultTemporal.  Halos travel K planes / rows / columns deep, so
  // every subdomain needs >= K owned points along each split axis.  y / z
  // splits (block decompositions) use the kernel's y / z update ranges and an
  // axis-ordered exchange that also fills the edge and corner ghosts a K-step
  // update reads.  Decided from the global decomposition so that every rank
  // agrees.  Auto depth: 3, for one subdomain and for x slabs alike.
  int K = cfg_.temporal >= 2 ? cfg_.temporal
          : kspec2_.multi_step() ? kspec2_.K
          : dt_ == DType::F64    ? kDefaultTemporal
                                 : kDefaultTemporalF32;
  // the sweep kernel: the lean kernel (stencil_tbl.hip; fp32 its packed-pair
  // form, stencil_tbp.hip); --kernel2 tlK:... / tsK:... picks a variant
  if (!kspec2_.multi_step()) kspec2_.kind = KernelSpec::TBL;
  kspec2_.K = K;
  int64_t min_n[3] = {INT64_MAX, INT64_MAX, INT64_MAX};
  for (const auto& sd : dec_.subs)
    for (int a = 0; a < 3; ++a) min_n[a] = std::min(min_n[a], sd.n[a]);
  const bool block = dims[1] > 1 || dims[2] > 1;
  const bool has_split = dims[0] * dims[1] * dims[2] > 1;
  bool fits = true;
  for (int a = 0; a < 3; ++a) fits &= dims[a] == 1 || min_n[a] >= K;
  tb_ = kspec_.kind != KernelSpec::Naive && (cfg_.temporal >= 2 || (cfg_.temporal == 0 && be_->is_gpu())) && fits;
  K_ = tb_ ? K : 1;
  for (int a = 0; a < 3; ++a) hd_[a] = xd_[a] = tb_ && dims[a] > 1 ? K : 1;
  ordered_halo_ = tb_ && block;
  // overlapped sweeps need a non-empty interior between the boundary layers
  // of every split axis; otherwise exchange first, then sweep
  bool thick = true;
  for (int a = 0; a < 3; ++a) thick &= dims[a] == 1 || min_n[a] >= 2 * K + 1;
  tb_overlap_ = tb_ && dims[0] * dims[1] * dims[2] > 1 && overlap_ && thick && (!block || cfg_.block_overlap);
  // lagged convergence check (third buffer, two residual-slot banks) keeps
  // the all-reduce + check off the critical path of the overlapped sweeps
  if (cfg_.lag == 1 && !(tb_overlap_ && 2 * K_ <= kResidualSlots))
    throw UsageError("--lag on needs overlapped temporally blocked sweeps of depth K <= " +
                     std::to_string(kResidualSlots / 2));
  lag_ = tb_overlap_ && 2 * K_ <= kResidualSlots && cfg_.lag != 0;
  nbuf_ = lag_ ? 3 : 2;
  // Long sweeps across halos: a step count n = a K + b (K+1) runs as a + b
  // sweeps instead of ending in a partial sweep of n mod K steps, whose HBM
  // pass costs nearly a full sweep (fp64 1022^3: K = 2 3.5 ms vs K = 3 3.6 ms)
  // — the driver's 20-step window at N > 1 is 6 x 3 + 2 otherwise.  Ghosts go
  // K+1 deep on split axes; only a long sweep exchanges K+1 planes.  Needs
  // K+1 owned points per split axis (2(K+1)+1 when overlapped), the K+1
  // kernel, and two banks of K+1 residual slots under the lagged check.
  // Whether a remainder actually runs as long sweeps is decided per run by
  // timing the sweeps at start-up (calibrate_remainders): on the 8-GPU slab
  // share a K+1 sweep costs 1.65-1.73x a K one.
  {
    bool ok = tb_ && has_split && cfg_.long_sweeps && K + 1 <= 6 && K + 1 <= kResidualSlots &&
              (!lag_ || 2 * (K + 1) <= kResidualSlots);
    for (int a = 0; a < 3; ++a) {
      ok &= dims[a] == 1 || min_n[a] >= K + 1;
      if (tb_overlap_) ok &= dims[a] == 1 || min_n[a] >= 2 * (K + 1) + 1;
    }
    if (ok && be_->is_gpu()) {
      KernelSpec ks;
      ks.kind = kspec2_.kind;
      ks.K = K + 1;
      ok = hip::lean_supported(dt_, ks);
    }
    long_halo_ = ok;
    if (long_halo_)
      for (int a = 0; a < 3; ++a)
        if (dims[a] > 1) hd_[a] = K + 1;
    slot_stride_ = K_ + (long_halo_ ? 1 : 0);
  }
  fake_allreduce_us_ = cfg_.fake_allreduce_us;
  // processes sharing this rank's GPU: the launcher's local world size over
  // the visible devices (one process hosting virtual ranks counts once)
  if (be_->is_gpu() && !comm_->all_local()) {
    int local = 0;
    for (const char* v : {"LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE", "MPI_LOCALNRANKS"}) {
      const char* e = std::getenv(v);
      if (e && *e) {
        local = std::atoi(e);
        break;
      }
    }
    const int ndev = std::max(1, hip_device_count());
    ranks_per_device_ = std::max(1, (local + ndev - 1) / ndev);
  }
  chain_ = comm_->ordered_collectives() && !comm_->all_local() && comm_->size() > 1;
  // a long x-slab interior (the 2-GPU 1024^3 share): the halo chain hides
  // under it with room to spare (no CU reservation)
  {
    int64_t least = INT64_MAX;
    for (const auto& sd : dec_.subs) least = std::min(least, (sd.n[0] - 2 * K_) * sd.n[1] * sd.n[2]);
    long_slab_ = tb_overlap_ && !block && least >= kLongSlabInterior && !comm_->all_local() && comm_->size() > 1;
  }
  // CU reservation for the overlapped schedule of a real multi-rank job
  // (RCCL or its phantom): the comm / boundary / check kernels must not queue
  // behind the interior sweep, which holds every CU (LDS / VGPR file full)
  {
    int n = cfg_.reserve_cus;
    if (n < 0) {
      n = multi_stream() && !comm_->all_local() && comm_->size() > 1 ? 8 : 0;
      // ...except under a long x-slab interior, which hides the halo chain
      // even when the comm kernels wait for a CU: RCCL's kernel (256 threads,
      // 140 VGPRs, 20 KB LDS; gpurun_out/r7t) cannot sit beside an interior
      // workgroup (16 waves x 112 VGPRs), so without the reservation it
      // starts at the next piece boundary, <= ~0.2 ms into the 2-GPU 1024^3
      // share's ~1.8 ms sweep.  That share (508 x 1022^2 interior points)
      // ran 4.8-7 % faster on all 256 CUs (proxy: 0.666-0.694 against
      // 0.715-0.736 ms/step, gpurun_out/r7s, r7u, r7v; 2 reserved CUs were
      // slower than 8), the 4-GPU share (250 planes) 1.3-11 % (0.385-0.415
      // against 0.421-0.435; the low end with the stand-in comm kernels in
      // RCCL's footprint, which wait for a CU as RCCL's does: r7t, r7w; at
      // 40 GB/s links 4-6 %, r8k).  The 8-GPU share keeps the reservation: its
      // chain runs as long as its interior, so an RCCL kernel that waits for a
      // CU would show, and the proxy models disagree (+1.2 % to -8.6 %, r8l).
      if (n > 0 && long_slab_) n = 0;
    }
    if (be_->is_gpu() && n > 0) be_->reserve_cus(n);
  }
  preflight_memory();

  for (int r : comm_->local_ranks()) {
    Local l;
    l.sd = dec_.subs[r];
    l.L = Layout::make(l.sd.n, (int64_t)esize_, hd_[0], hd_[1], hd_[2]);
    for (int b = 0; b < nbuf_; ++b) l.field[b] = be_->alloc(l.L.bytes());
    for (int a = 0; a < 3; ++a) {
      l.owned.lo[a] = 0;
      l.owned.hi[a] = l.sd.n[a];
    }
    Decomposition::split_interior(l.sd, &l.interior, &l.shell);
    const bool lo = l.sd.has_neighbor(Face::Left), hi = l.sd.has_neighbor(Face::Right);
    l.ux[0] = lo ? -(K_ - 1) : 0;
    l.ux[1] = l.sd.n[0] + (hi ? K_ - 1 : 0);
    // y / z update ranges reach into deep halos only where there is one
    for (int a = 1; a < 3; ++a) {
      int64_t* u = a == 1 ? l.uy : l.uz;
      const bool nlo = l.sd.has_neighbor(static_cast<Face>(2 * a));
      const bool nhi = l.sd.has_neighbor(static_cast<Face>(2 * a + 1));
      u[0] = nlo && hd_[a] > 1 ? -(K_ - 1) : 0;
      u[1] = l.sd.n[a] + (nhi && hd_[a] > 1 ? K_ - 1 : 0);
    }
    // interior / boundary pieces of the overlapped sweeps of depth d
    auto pieces = [&](int64_t d, Box* interior, std::vector<Box>* boundary) {
      *interior = l.owned;
      boundary->clear();
      if (!tb_overlap_) return;
      // interior: the owned box minus a d-thick layer on every face with a
      // neighbour (its d-step update reads no ghost).  Boundary pieces, an
      // onion: the d-thick layers of axis a span the interior range of the
      // axes before a and the full range of the axes after it — disjoint,
      // and together with the interior they tile the owned box.
      bool nb[3][2];
      for (int a = 0; a < 3; ++a)
        for (int e = 0; e < 2; ++e) nb[a][e] = hd_[a] > 1 && l.sd.has_neighbor(static_cast<Face>(2 * a + e));
      // Layer thickness per axis.  x: d (the y-marching thin-slab tiles, the
      // halo-depth bookkeeping of long sweeps).  y / z: one tile stride (the
      // rows / columns a sweep tile stores: TY - 2d, 64 V - 2d) where the
      // subdomain leaves an interior at least that thick — a d-thin layer
      // stores d of the tile's TY rows or 64 V columns, e.g. 3 of 120 columns
      // for fp32 pairs: a 1018^2 z layer took 0.77 ms against ~0.03 ms of
      // interior work (phantom 2x2x2 trace, round 4)
      int64_t t[3] = {d, d, d};
      if (cfg_.tile_layers) {
        const KernelSpec rs = kspec2_.resolved(dt_);
        const int64_t want[3] = {d, (int64_t)rs.WY * rs.R - 2 * d, 64 * (int64_t)std::max(1, rs.V) - 2 * d};
        for (int a = 1; a < 3; ++a) {
          const int64_t ta = std::max(d, want[a]);
          const int sides = (int)nb[a][0] + (int)nb[a][1];
          if (sides && l.sd.n[a] - sides * ta >= std::max(ta, 2 * d + 1)) t[a] = ta;
        }
      }
      for (int a = 0; a < 3; ++a) {
        if (nb[a][0]) interior->lo[a] = t[a];
        if (nb[a][1]) interior->hi[a] = l.sd.n[a] - t[a];
      }
      for (int a = 0; a < 3; ++a)
        for (int side = 0; side < 2; ++side) {
          if (!nb[a][side]) continue;
          Box b = l.owned;
          for (int c = 0; c < a; ++c) {
            b.lo[c] = interior->lo[c];
            b.hi[c] = interior->hi[c];
          }
          b.lo[a] = side ? l.sd.n[a] - t[a] : 0;
          b.hi[a] = b.lo[a] + t[a];
          boundary->push_back(b);
        }
    };
    pieces(K_, &l.tb_interior, &l.tb_boundary);
    if (long_halo_) {
      pieces(K_ + 1, &l.tb_interior_long, &l.tb_boundary_long);
    } else {  // long sweeps of a single subdomain (no ghosts to widen into)
      l.tb_interior_long = l.tb_interior;
      l.tb_boundary_long = l.tb_boundary;
    }
    local_.push_back(l);
  }
  setup_faces();
  dstate_ = static_cast<DeviceState*>(be_->alloc(sizeof(DeviceState)));
  hstate_ = static_cast<DeviceState*>(be_->alloc_host(2 * sizeof(DeviceState)));
  std::memset(hstate_, 0, 2 * sizeof(DeviceState));
  for (int i = 0; i < EV_COUNT; ++i) cur_ev_[i] = ev_[i] = be_->event_create();
}

Solver::~Solver() {
  try {
    be_->sync_all();
  } catch (...) {
  }
  destroy_graphs();
  for (auto& e : ev_)
    if (e) be_->event_destroy(e);
  for (auto& e : cap_pool_) be_->event_destroy(e);
  for (auto& e : tev_)
    if (e) be_->event_destroy(e);
  for (auto& e : prof_ev_) be_->event_destroy(e);
  for (auto& l : local_) {
    for (auto* f : l.field)
      if (f) be_->release(f);
    for (auto& io : l.faces) {
      be_->release(io.sendbuf);
      be_->release(io.recvbuf);
    }
  }
  be_->release(dstate_);
  if (rstate_) be_->release(rstate_);
  be_->release_host(hstate_);
  comm_.reset();  // communicators before the device
}

// Refuses a configuration whose buffers do not fit before allocating any of
// them: nbuf_ fields (with K-deep halos) per local rank plus the y / z face
// staging buffers, against the backend's free memory less a reserve for RCCL
// channels, code objects and scratch (--mem-reserve-gb, default 2;
// --no-mem-preflight skips the check).  A 4096^3 fp32 grid on 2x2x2 GPUs
// plans 3 x 34.6 GB per rank; 8192^3 fp32 on 2x2x2 (3 x 275 GB) is refused.
void Solver::preflight_memory() {
  planned_bytes_ = 0;
  for (int r : comm_->local_ranks()) {
    const Subdomain& sd = dec_.subs[r];
    const Layout L = Layout::make(sd.n, (int64_t)esize_, hd_[0], hd_[1], hd_[2]);
    planned_bytes_ += (std::size_t)nbuf_ * L.bytes();
    if (comm_->all_local()) continue;
    for (int a = 1; a < 3; ++a)  // packed y / z faces: a send and a receive buffer each
      for (int side = 0; side < 2; ++side) {
        if (!sd.has_neighbor(static_cast<Face>(2 * a + side))) continue;
        std::size_t e = (std::size_t)hd_[a] * esize_;
        for (int b = 0; b < 3; ++b)
          if (b != a) e *= (std::size_t)(sd.n[b] + 2 * hd_[b]);
        planned_bytes_ += 2 * e;
      }
  }
  if (!be_->mem_info(&mem_free_before_, &mem_total_)) return;
  if (!cfg_.mem_preflight) return;
  const double reserve = cfg_.mem_reserve_gb * 1e9;
  if ((double)planned_bytes_ + reserve > (double)mem_free_before_) {
    const auto& n = cfg_.n;
    HEAT3D_THROW("memory preflight: the " << n[0] << "x" << n[1] << "x" << n[2] << " " << dtype_name(dt_)
                 << " grid on " << comm_->size() << " rank(s) needs " << planned_bytes_ / 1e9 << " GB on this "
                 << (be_->is_gpu() ? "GPU" : "host") << " (" << comm_->local_ranks().size() << " local subdomain(s) x "
                 << nbuf_ << " field buffers + face staging) plus a " << reserve / 1e9 << " GB reserve, but only "
                 << mem_free_before_ / 1e9 << " of " << mem_total_ / 1e9
                 << " GB are free; use more ranks" << (dt_ == DType::F64 ? ", fp32" : "")
                 << (nbuf_ == 3 ? ", or two field buffers (--lag off)" : ""));
  }
}

bool Solver::is_root() const {
  for (const auto& l : local_)
    if (l.sd.rank == 0) return true;
  return false;
}

void Solver::setup_faces() {
  has_halo_ = false;
  for (auto& l : local_) {
    for (int f = 0; f < kNumFaces; ++f) {
      const Face face = static_cast<Face>(f);
      if (!l.sd.has_neighbor(face)) continue;
      has_halo_ = true;
      FaceIO io;
      io.face = face;
      io.peer = l.sd.neighbors[f];
      const int a = face_axis(face), side = face_side(face);
      for (int dv = 0; dv < 2; ++dv) {
        // exchange depth: the regular one, or the ghost depth (K+1 with long_halo_)
        auto depth = [&](int b) { return dv ? hd_[b] : xd_[b]; };
        FaceGeom& fg = io.g[dv];
        for (int b = 0; b < 3; ++b) {
          fg.send_box.lo[b] = fg.recv_box.lo[b] = 0;
          fg.send_box.hi[b] = fg.recv_box.hi[b] = l.sd.n[b];
        }
        const int64_t dep = depth(a);
        fg.send_box.lo[a] = side ? l.sd.n[a] - dep : 0;
        fg.send_box.hi[a] = fg.send_box.lo[a] + dep;
        fg.recv_box.lo[a] = side ? l.sd.n[a] : -dep;
        fg.recv_box.hi[a] = fg.recv_box.lo[a] + dep;
        if (ordered_halo_) {
          // axis-ordered exchange (x, then y, then z): a face of axis a also
          // carries the deep ghosts of the axes before it, which the earlier
          // phases have filled, so edges and corners arrive in the right order
          for (int b = 0; b < a; ++b) {
            const int64_t elo = l.sd.has_neighbor(static_cast<Face>(2 * b)) ? depth(b) : 0;
            const int64_t ehi = l.sd.has_neighbor(static_cast<Face>(2 * b + 1)) ? depth(b) : 0;
            fg.send_box.lo[b] = fg.recv_box.lo[b] = -elo;
            fg.send_box.hi[b] = fg.recv_box.hi[b] = l.sd.n[b] + ehi;
          }
        }
        if (a == 0) {
          // x faces: whole planes (ghost rows and padding included) are
          // contiguous; the neighbour across an x face has the same ny, nz and
          // therefore the same strides.
          fg.send_off = l.L.plane_offset(fg.send_box.lo[0]);
          fg.recv_off = l.L.plane_offset(fg.recv_box.lo[0]);
          fg.elems = dep * l.L.sx;
        } else {
          fg.elems = fg.send_box.volume();
        }
      }
      if (comm_->all_local()) {
        for (std::size_t q = 0; q < local_.size(); ++q)
          if (local_[q].sd.rank == io.peer) io.peer_local = (int)q;
        HEAT3D_CHECK(io.peer_local >= 0, "local neighbour not found");
      } else if (a == 0) {
        io.contiguous = true;
      } else {
        io.sendbuf = be_->alloc(io.g[1].elems * esize_);
        io.recvbuf = be_->alloc(io.g[1].elems * esize_);
      }
      l.faces.push_back(io);
    }
  }
  if (!has_halo_) overlap_ = false;  // nothing to overlap with
}

InitParams Solver::init_params(const Local& l) const {
  InitParams p;
  p.L = l.L;
  for (int a = 0; a < 3; ++a) {
    p.gstart[a] = l.sd.gstart[a];
    p.N[a] = dec_.N[a];
    p.h[a] = phys_.h[a];
  }
  return p;
}

void Solver::ev_record(int id, StreamId s) {
  if (capturing_) {
    // inside a stream capture every record gets a fresh event (the HIP
    // runtime does not tolerate re-recording one event within a capture)
    HEAT3D_CHECK(cap_next_ < cap_pool_.size(), "capture event pool exhausted");
    cur_ev_[id] = cap_pool_[cap_next_++];
  } else {
    cur_ev_[id] = ev_[id];
  }
  be_->record(cur_ev_[id], s);
  ev_valid_[id] = true;
}

void Solver::ev_wait(StreamId s, int id) {
  if (ev_valid_[id]) be_->wait(s, cur_ev_[id]);
}

void Solver::initialize() {
  be_->sync_all();
  destroy_graphs();
  pending_.valid = false;
  init_fields();
  sweep_costs_.clear();
  if (pick_sweep_form()) {  // re-timed from the lean form on every initialisation
    KernelSpec lean;
    lean.kind = kspec2_.kind;
    lean.K = K_;
    kspec2_ = lean;
  }
  rl_ = false;
  for (bool& b : rl_d_) b = false;
  tune_schedules();
  calibrate_remainders();
  // the sweep form is final: its last-residual variant, where one exists
  // the sweep shapes are final: their last-residual variants, where they exist
  if (residual_last_ok())
    for (int Kp = 2; Kp <= K_ + 1 && Kp < 8; ++Kp) {
      // the timed winner where it is a last-residual variant, else the
      // depth's shape in that form
      const bool picked = (rl_pick_[Kp].O & kResidualLastOnly) != 0;
      ks_last_[Kp] = picked ? rl_pick_[Kp] : last_only(spec_for_depth(Kp));
      // (block decompositions: long sweeps keep every residual, see long_major_)
      rl_d_[Kp] = hip::lean_supported(dt_, ks_last_[Kp]) && !(ordered_halo_ && Kp > K_);
    }
  rl_ = rl_d_[K_];
  reset_state();
  canary_stream_graphs();
}

void Solver::init_fields() {
  for (auto& l : local_) {
    InitParams p = init_params(l);
    for (int b = 0; b < nbuf_; ++b) {
      p.field = l.field[b];
      be_->init_field(dt_, p, kCompute);
    }
  }
}

void Solver::reset_state() {
  DeviceState hs;
  std::memset(&hs, 0, sizeof(hs));
  for (auto& r : hs.residual) r = kResidualInitBits;
  hs.norm = 1.0;  // heat3D.cu:323-324 (norm = 1 until iteration 0 sets it)
  hs.eps = cfg_.eps;
  hs.iter = 0;
  hs.conv_iter = -1;
  hs.hist_cap = 1024;
  // a device-side graph wait longer than the watchdog is a broken dependency
  // or a stalled peer: the kernel flags it instead of holding the GPU
  hs.wait_ticks = (uint64_t)(cfg_.watchdog_s * 1e8);
  std::memcpy(hstate_, &hs, sizeof(hs));
  be_->copy(dstate_, hstate_, sizeof(DeviceState), CopyKind::H2D, kCompute);
  be_->sync(kCompute);
  issued_ = 0;
  cur_ = 0;
  nsweep_ = 0;
  last_kind_ = 0;
  last_bnd_ = 0;
  segs_.clear();
  seg_head_ = 0;
  sg_unchecked_ = false;
  if (!cfg_.restart.empty()) load_checkpoint(cfg_.restart);
  // make every pipeline event valid (complete) before the first iteration
  for (int i = 0; i < EV_COUNT; ++i) ev_valid_[i] = false;
  for (int p = 0; p < 2; ++p) {
    ev_record(EV_INT + p, kCompute);
    ev_record(EV_BND + p, kComm);
    ev_record(EV_CHK + p, kReduce);
  }
  be_->sync_all();
  comm_->barrier(*be_);
}

void Solver::set_wait_timeout(double seconds) {
  const uint64_t t = (uint64_t)(seconds * 1e8);  // 100 MHz real-time clock
  hstate_->wait_ticks = t;
  be_->copy(reinterpret_cast<char*>(dstate_) + offsetof(DeviceState, wait_ticks), &hstate_->wait_ticks,
            sizeof(uint64_t), CopyKind::H2D, kCompute);
  be_->sync(kCompute);
}

void Solver::check_graph_fault() {
  if (!sg_unchecked_) return;
  sg_unchecked_ = false;
  int32_t f = 0;
  be_->copy(&f, reinterpret_cast<char*>(dstate_) + offsetof(DeviceState, fault), sizeof(int32_t), CopyKind::D2H,
            kCompute);
  be_->sync(kCompute);
  HEAT3D_CHECK(f != 2, "a device-side wait of a per-stream hipGraph timed out after "
                           << cfg_.watchdog_s << " s (broken dependency or a stalled peer)");
}

// Per-stream graphs replace cross-stream events by spinning one-wave wait
// kernels on the consumer's stream.  They hold only while each stream keeps a
// hardware queue of its own: a wait queued behind the work it waits for on a
// shared queue never ends (the 8-ranks-on-one-GPU rehearsal hung that way,
// round 5).  Nothing in HIP reports the queue mapping, so the schedule is
// tried once, at start-up, with a short timeout, and kept only if it ran.
void Solver::canary_stream_graphs() {
  sg_note_.clear();
  if (!multi_stream() || !be_->supports_graphs()) {
    sg_state_ = "n/a";
    return;
  }
  if (!graphs_allowed()) {
    sg_state_ = sg_fallback_ ? "fallback" : "off";
    return;
  }
  if (cfg_.graph_canary_s <= 0) {
    sg_state_ = "unverified";
    return;
  }
  const int64_t cyc = tb_ ? (int64_t)K_ * (nbuf_ == 3 ? 6 : 2) : (nbuf_ == 3 ? 6 : 2);
  const int G = graph_len_for(cyc);
  if (G <= 0) {
    sg_state_ = "unverified";
    return;
  }
  set_wait_timeout(cfg_.graph_canary_s);
  force_eager_ = true;
  comm_->barrier(*be_);
  double t0 = now_s();
  run_chunk(G);
  be_->sync_all();
  const double eager = now_s() - t0;
  force_eager_ = false;
  prepare_steps(G);
  const int64_t launches = graph_launches_;
  comm_->barrier(*be_);
  // The device-side waits give up after --graph-canary, but RCCL's own
  // kernels wait for their peers without a limit: on a GPU whose hardware
  // queues are oversubscribed (8 ranks of a rehearsal on one device) a peer's
  // transfer kernel may never be scheduled behind a spinning wait, and the
  // replay never ends (round 6, gpurun_out/r6f).  So the host bounds it too:
  // past the limit the communicators are aborted (RCCL's kernels exit on the
  // abort flag, the waits on their timeout) and initialize() throws; the
  // vote below is bounded the same way for ranks whose replay ended while a
  // peer's did not.  HeatSolver.initialize() then rebuilds the solver with
  // the graphs off (a new communicator), every rank alike.
  const double host_limit = std::max(10.0 + 4.0 * cfg_.graph_canary_s, 20.0 * eager);
  auto deadlock = [&](const char* where) {
    H3D_TRACE("canary: " << where << " after " << host_limit << " s: aborting the communicators");
    // ncclCommAbort itself can hang on such a GPU (8 processes of a one-GPU
    // rehearsal with the graphs forced on: it never returned, gpurun_out/r6h):
    // run it on a helper thread and, if it does not return, end the process
    // with a clear error instead of hanging the job
    std::atomic<bool> aborted{false};
    std::thread t([&] {
      comm_->abort();
      aborted = true;
    });
    const double ta = now_s();
    while (!aborted && now_s() - ta < 10.0) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    if (!aborted) {
      std::fprintf(stderr,
                   "heat3d: stream-graph canary deadlock: the per-stream hipGraph replay %s within %.1f s and "
                   "ncclCommAbort did not return in 10 s (oversubscribed GPU?); exiting — rerun with "
                   "--stream-graphs off\n",
                   where, host_limit);
      std::fflush(stderr);
      std::_Exit(86);
    }
    t.join();
    H3D_TRACE("canary: communicators aborted");
    const bool drained = be_->sync_all_for(2.0 * cfg_.graph_canary_s + 5.0);
    H3D_TRACE("canary: streams " << (drained ? "drained" : "still busy"));
    HEAT3D_THROW("stream-graph canary deadlock: the per-stream hipGraph replay " << where << " within " << host_limit
                 << " s (oversubscribed hardware queues?); communicators aborted; rerun with --stream-graphs off");
  };
  H3D_TRACE("canary: eager cycle " << eager * 1e3 << " ms, graph captured; replaying (host limit " << host_limit << " s)");
  t0 = now_s();
  run_chunk(G);
  if (!be_->sync_all_for(host_limit)) deadlock("did not finish");
  H3D_TRACE("canary: replay done in " << (now_s() - t0) * 1e3 << " ms");
  const double graph = now_s() - t0;
  sg_unchecked_ = false;
  be_->copy(hstate_, dstate_, offsetof(DeviceState, hist), CopyKind::D2H, kCompute);
  be_->sync(kCompute);
  const bool timed_out = hstate_->fault == 2;
  const bool replayed = graph_launches_ > launches;
  const bool slow = graph > 2.0 * eager + 1e-3;
  // one decision for the job: the ranks' schedules must stay the same kind
  // (their collectives pair up either way, but a mixed job has no use)
  unsigned long long vote = (timed_out ? 1ull << 40 : 0ull) + (slow ? 1ull << 20 : 0ull) + (replayed ? 0ull : 1ull);
  if (!comm_->all_local() && comm_->size() > 1) {
    void* d = be_->alloc(8);
    be_->copy(d, &vote, 8, CopyKind::H2D, kReduce);
    comm_->allreduce(d, 1, RedType::U64, RedOp::Sum, *be_, kReduce);
    be_->copy(&vote, d, 8, CopyKind::D2H, kReduce);
    const bool ok = be_->sync_all_for(host_limit);
    if (ok) be_->release(d);
    if (!ok) deadlock("vote did not complete (a peer's replay hung)");
  }
  std::ostringstream os;
  os.setf(std::ios::fixed);
  os.precision(3);
  os << G << " iterations: graphs " << graph * 1e3 << " ms, eager " << eager * 1e3 << " ms";
  if (vote >> 40) os << "; " << (vote >> 40) << " rank(s) timed out in a device-side wait";
  if ((vote >> 20) & 0xfffff) os << "; " << ((vote >> 20) & 0xfffff) << " rank(s) replayed > 2x eager";
  if (vote & 0xfffff) os << "; " << (vote & 0xfffff) << " rank(s) did not replay a graph";
  sg_note_ = os.str();
  if (vote) {
    sg_fallback_ = true;
    sg_state_ = "fallback";
    destroy_graphs();
    if (!cfg_.quiet && is_root())
      std::fprintf(stderr, "heat3d: per-stream hipGraph canary failed (%s); the overlapped schedule runs eagerly\n",
                   sg_note_.c_str());
  } else {
    sg_state_ = "on";
  }
  // back to iteration 0 (reset_state restores the watchdog-long wait timeout)
  init_fields();
  reset_state();
}

// Time the x-schedule candidates of every interior sweep shape this run will
// launch (hip::tune_x_schedule) before the first iteration, on the freshly
// initialised fields: each candidate computes sweep 0 of the interior box
// into the next buffer without residual state, which the first real sweep
// overwrites with the same values.  The chosen schedules then serve every
// eager launch and every graph capture of the run.
void Solver::tune_schedules() {
  // auto: only where a sweep runs alone as it is timed here.  Under the
  // overlapped multi-rank schedule the interior shares the GPU with the halo
  // chain, and a standalone timing did not predict it: the phantom 8-GPU
  // share's interior timed 56-column / 61-plane pieces 12% faster alone, then
  // ran 9% slower than the model's choice in the schedule (same ms per step;
  // profiles/rank_proxy_r03.md)
  const bool on = cfg_.autotune > 0 || (cfg_.autotune < 0 && !has_halo_ && local_.size() == 1);
  if (!on || !tb_ || !be_->is_gpu()) return;
  std::vector<KernelSpec> specs{kspec2_};
  if (pick_sweep_form()) specs.push_back(pair_form());
  if ((!has_halo_ || long_halo_) && cfg_.long_sweeps && K_ + 1 <= 6 && K_ + 1 <= kResidualSlots) {
    KernelSpec ks;
    ks.kind = kspec2_.kind;
    ks.K = K_ + 1;
    if (hip::lean_supported(dt_, ks)) specs.push_back(ks);
  }
  // the last-residual variants of those: kernels of their own, whose
  // schedules are timed (and looked up) separately
  if (residual_last_ok()) {
    const std::size_t nf = specs.size();
    for (std::size_t i = 0; i < nf; ++i) {
      const KernelSpec r = last_only(specs[i]);
      if (hip::lean_supported(dt_, r)) specs.push_back(r);
    }
  }
  for (const KernelSpec& ks : specs) {
    const int Kp = ks.K;
    for (auto& l : local_) {
      const Box& box = Kp > K_ ? l.tb_interior_long : l.tb_interior;
      if (box.empty()) continue;
      StencilParams sp;
      sp.in = l.field[0];
      sp.out = l.field[nxt(0)];
      sp.L = l.L;
      sp.box = box;
      for (int a = 0; a < 3; ++a) sp.D[a] = phys_.D[a];
      sp.state = nullptr;
      sp.cu_reserved = be_->reserved_cus();
      sp.tune = true;
      auto shrink = [&](const int64_t (&u)[2], int64_t n, int64_t (&o)[2]) {
        o[0] = u[0] < 0 ? -(Kp - 1) : u[0];
        o[1] = u[1] > n ? n + Kp - 1 : u[1];
      };
      shrink(l.ux, l.sd.n[0], sp.ux);
      shrink(l.uy, l.sd.n[1], sp.uy);
      shrink(l.uz, l.sd.n[2], sp.uz);
      be_->sweep(dt_, sp, ks, kCompute);
    }
  }
  be_->sync(kCompute);
}

// Remainder policy.  A step count n = a K + r (0 < r < K) either ends in a
// partial sweep of r steps (r = 1: a single step) or runs r of its sweeps as
// long sweeps of K+1 steps: long costs r (T_{K+1} - T_K) more sweep time,
// partial costs T_r.  Which is cheaper depends on the box: on one GPU's
// 1022^3 a K = 2 sweep takes 95% of a K = 3 one (3.5 vs 3.7 ms; long wins),
// on the 8-GPU slab share's 122-plane interior the K = 4 sweep takes 1.73x
// the K = 3 one (936 vs 540 us: its 36-row tiles need 2.8 rounds of
// workgroups against 1.8) while K = 2 takes 0.96x (partial wins).  So each
// rank times its interior sweeps once at start-up (idempotent sweeps into
// the next buffer, no residual state, as tune_schedules) and the ranks agree
// by vote: long for remainder r only where every rank found it cheaper.
KernelSpec Solver::spec_for_depth(int Kp) const {
  if (Kp == K_) return kspec2_;
  if (Kp >= 0 && Kp < 8 && depth_set_[Kp]) return depth_spec_[Kp];
  KernelSpec ks;
  ks.kind = kspec2_.kind;
  ks.K = Kp;
  return ks;
}

// Sweep form of a single-subdomain fp64 run: the one-value-per-lane lean
// kernel or its 16-byte pair form (stencil_tbp.hip), whichever the start-up
// timing finds faster on this box.  Same box, driver window (1 GPU, 1024^3,
// 20 / 5): pair 851.5-853.5 against lean 839.6-842.4 GLUPS, where the
// kernel-level timing of round 5's first boxes had the pair form 1.5% slower
// (profiles/fp64_pairs_r05.md).  Only where the sweeps run alone as timed;
// under the overlapped multi-rank schedule the standalone timing picked the
// pairs and they ran no faster there; on the 2-GPU share, whose interior
// hides its halo chain, the pair form timed 1 % faster and ran the same
// (0.6775-0.6793 against 0.6776-0.6804 ms/step, gpurun_out/r7y).
bool Solver::pick_sweep_form() const {
  if (!tb_ || !be_->is_gpu() || dt_ != DType::F64 || has_halo_ || local_.size() != 1 || cfg_.kernel2 != "auto" ||
      kspec2_.kind != KernelSpec::TBL)
    return false;
  return hip::lean_supported(dt_, pair_form());
}

KernelSpec Solver::pair_form() const {
  KernelSpec p;
  p.kind = kspec2_.kind;
  p.K = K_;
  p.V = 2;
  return p;
}

void Solver::calibrate_remainders() {
  long_major_ = false;
  for (auto& k : rl_pick_) k = KernelSpec{};
  long_rem_ = ~0u;
  for (bool& d : depth_set_) d = false;
  if (!tb_ || cfg_.long_sweeps == 0) {
    long_rem_ = 0;
    return;
  }
  if (cfg_.long_sweeps == 1 || (cfg_.long_sweeps < 0 && !be_->is_gpu()) || (has_halo_ && !long_halo_) ||
      K_ + 1 > 6)
    return;
  if (be_->is_gpu()) {
    KernelSpec kl;
    kl.kind = kspec2_.kind;
    kl.K = K_ + 1;
    if (!hip::lean_supported(dt_, kl)) return;
  }
  struct Events {  // released on every exit (a refused kernel variant throws)
    Backend* be;
    Event a, b;
    ~Events() {
      be->event_destroy(a);
      be->event_destroy(b);
    }
  } ev{be_.get(), be_->event_create(), be_->event_create()};
  Event e0 = ev.a, e1 = ev.b;
  // Kp = 1: a single step of the owned box; else a sweep of depth Kp
  auto launch = [&](int Kp, const KernelSpec& ks) {
    for (auto& l : local_) {
      StencilParams sp;
      sp.in = l.field[0];
      sp.out = l.field[nxt(0)];
      sp.L = l.L;
      for (int a = 0; a < 3; ++a) sp.D[a] = phys_.D[a];
      sp.state = nullptr;
      sp.cu_reserved = be_->reserved_cus();
      if (Kp == 1) {
        sp.box = l.owned;
        be_->stencil(dt_, sp, kspec_, kCompute);
        continue;
      }
      sp.box = Kp > K_ ? l.tb_interior_long : l.tb_interior;
      if (sp.box.empty()) continue;
      auto shrink = [&](const int64_t (&u)[2], int64_t nn, int64_t (&o)[2]) {
        o[0] = u[0] < 0 ? -(Kp - 1) : u[0];
        o[1] = u[1] > nn ? nn + Kp - 1 : u[1];
      };
      shrink(l.ux, l.sd.n[0], sp.ux);
      shrink(l.uy, l.sd.n[1], sp.uy);
      shrink(l.uz, l.sd.n[2], sp.uz);
      be_->sweep(dt_, sp, ks, kCompute);
    }
  };
  // candidates: the K and K+1 sweeps, a single step, the partial sweeps;
  // fp64 K = 2 in three tile shapes: 80-row tiles (fewer halo rows per stored
  // one), 48-row ones (a 122-plane slab share on 248 CUs takes 252 of the
  // tall tiles = two rounds, 450 short ones also two: the short ones won
  // there, 0.52 against 0.70 ms) and 48 x 128 pair tiles (stencil_tbp.hip:
  // 624 against 584 GLUPS on 1022^3; a 1022^2 face is 216 of them, one round)
  struct Cand {
    int Kp;
    KernelSpec ks;
    std::string name;
    KernelSpec form;  // the sweep shape the candidate stands for (it times the variant that runs)
  };
  // sweeps after iteration 0 run a shape's last-residual variant where the
  // monotone check is on: the shapes are timed (and compared) as they run
  const bool rl_forms = residual_last_ok();
  auto as_run = [&](const KernelSpec& f) {
    if (!rl_forms) return f;
    const KernelSpec r = last_only(f);
    return hip::lean_supported(dt_, r) ? r : f;
  };
  std::vector<Cand> cands{{K_, as_run(kspec2_), "sweep" + std::to_string(K_), kspec2_},
                          {K_ + 1, as_run(spec_for_depth(K_ + 1)), "sweep" + std::to_string(K_ + 1),
                           spec_for_depth(K_ + 1)}};
  // fp64 K = 4 in 48-row tiles of 12 waves (167 VGPRs in the last-residual
  // form): the fastest long sweep on one GPU (1022^3 / 510^3 kernel level 906 /
  // 846 against 886-892 / 824 for 36-row tiles, gpurun_out/r6k4)
  if (dt_ == DType::F64 && K_ == 3 && kspec2_.kind == KernelSpec::TBL && cfg_.kernel2 == "auto" && rl_forms) {
    // (the every-residual form spills: iteration 0's sweep and the replay of
    // one that converged run the default K + 1 shape)
    const KernelSpec t = KernelSpec::parse("tl4:1:4:1:12:0:3:66");
    if (hip::lean_supported(dt_, t))
      cands.push_back({K_ + 1, t, "sweep" + std::to_string(K_ + 1) + "[" + t.str() + "]", spec_for_depth(K_ + 1)});
  }
  const bool pick_form = pick_sweep_form();
  if (pick_form) {
    const KernelSpec pr = as_run(pair_form());
    cands.push_back({K_, pr, "sweep" + std::to_string(K_) + "[" + pr.resolved(dt_).str() + "]", pair_form()});
    KernelSpec pl = pair_form();  // and the pair form of the long sweep
    pl.K = K_ + 1;
    if (hip::lean_supported(dt_, pl))
      cands.push_back({K_ + 1, as_run(pl), "sweep" + std::to_string(K_ + 1) + "[" + pl.resolved(dt_).str() + "]", pl});
  }
  for (int r = 1; r < K_; ++r) {
    if (r == 2 && dt_ == DType::F64 && kspec2_.kind == KernelSpec::TBL && be_->is_gpu()) {
      for (const char* v : {"tl2:1:5:1:16:0:3:2", "tl2:1:3:1:16:0:3:2", "tl2:2:6:1:8:0:3:2"}) {
        const KernelSpec ks = KernelSpec::parse(v);
        if (hip::lean_supported(dt_, ks)) cands.push_back({2, as_run(ks), std::string("sweep2[") + v + "]", ks});
      }
      continue;
    }
    const KernelSpec base = r == 1 ? kspec_ : spec_for_depth(r);
    cands.push_back({r, r == 1 ? base : as_run(base), r == 1 ? std::string("step") : "sweep" + std::to_string(r), base});
  }
  // the GPU is cold here (initialisation, no sweeps yet): keep it busy with
  // regular sweeps for >= 30 ms before timing, then take the best of two
  // interleaved rounds per candidate (a cold first timing inflated the
  // 8-GPU share's K = 3 sweep by 20% and flipped the decision)
  std::vector<double> best(cands.size(), 1e30);
  {
    be_->record(e0, kCompute);
    launch(K_, kspec2_);
    be_->record(e1, kCompute);
    be_->sync(kCompute);
    const double one = std::max(1e-3, (double)be_->elapsed_ms(e0, e1));
    const int warm = std::max(1, std::min(200, (int)std::ceil(30.0 / one)));
    for (int i = 0; i < warm; ++i) launch(K_, kspec2_);
  }
  constexpr int reps = 3;
  for (int round = 0; round < 2; ++round)
    for (std::size_t c = 0; c < cands.size(); ++c) {
      be_->record(e0, kCompute);
      for (int i = 0; i < reps; ++i) launch(cands[c].Kp, cands[c].ks);
      be_->record(e1, kCompute);
      be_->sync(kCompute);
      best[c] = std::min(best[c], (double)be_->elapsed_ms(e0, e1) / reps);
    }
  // per depth: the fastest candidate (a rank-local kernel choice: the halo
  // of a partial sweep does not depend on its tile shape)
  std::vector<double> cost(K_ + 2, 1e30);
  for (std::size_t c = 0; c < cands.size(); ++c) {
    sweep_costs_.push_back({cands[c].name, best[c]});
    const int Kp = cands[c].Kp;
    if (best[c] < cost[Kp]) {
      cost[Kp] = best[c];
      if (Kp > 1 && Kp < 8) rl_pick_[Kp] = cands[c].ks;  // the variant that runs (last residual or not)
      if (Kp != K_ && Kp > 1) {
        depth_spec_[Kp] = cands[c].form;
        depth_set_[Kp] = true;
      }
      if (Kp == K_ && pick_form) kspec2_ = cands[c].form;  // the faster sweep form (pick_sweep_form)
    }
  }
  for (int Kp = 2; Kp < K_; ++Kp)
    if (cands.size() && cost[Kp] < 1e30 && std::count_if(cands.begin(), cands.end(), [&](const Cand& c) {
          return c.Kp == Kp;
        }) > 1)
      sweep_costs_.push_back({"sweep" + std::to_string(Kp), cost[Kp]});
  const double tk = cost[K_], tl = cost[K_ + 1];
  // long-major: where a K+1 sweep costs less per step than a K one (one
  // subdomain: the last-residual K = 4 sweep at 1022^3, 4.18 against 3.29 ms
  // for K = 3; not the 8-GPU slab share, whose 122-plane interior packs K + 1
  // tiles badly), step counts run as many long sweeps as they can
  // (long_sweeps_for)
  // (with halos the same 15 % margin as the remainder vote below; every rank
  // must agree: slot 0 of the vote)
  // (not block decompositions: a converged long sweep of a 2x2x2 run rolled
  // back to a different field under it on the GPU — gpurun_out/r6v5, and with
  // every residual in the long sweeps too, r6lb — while the CPU backend's
  // 2x2x2 / 1x2x2 long-major runs were bitwise; not yet explained, so blocks
  // keep K-step sweeps)
  long_major_ = (!has_halo_ || long_halo_) && !ordered_halo_ && tl < 1e30 &&
                (cfg_.long_sweeps == 3 || tl / (K_ + 1) * (has_halo_ ? 1.15 : 1.0) < tk / K_);
  // votes for the partial sweep, one slot per remainder; the ranks agree on
  // the max: long only where no rank found the partial sweep cheaper (the
  // halo depth of every exchange must match between neighbours)
  // With halos the timed interiors understate a long sweep: it also moves
  // (K+1)-deep halos and thicker boundary slabs.  On the 8-GPU slab share
  // (phantom rank, driver window) long sweeps for r = 2 timed 5 % cheaper than
  // the partial one (0.434 vs 0.456 ms) and ran the window 7 % slower (0.2400
  // against 0.2234 ms/step, gpurun_out/r6o): a long remainder must win by
  // 15 % there.
  const double margin = has_halo_ ? 1.15 : 1.0;
  std::vector<unsigned long long> partial(K_, 0);
  for (int r = 1; r < K_; ++r) partial[r] = r * (tl - tk) * margin < cost[r] ? 0 : 1;
  partial[0] = long_major_ ? 0 : 1;
  if (!comm_->all_local() && comm_->size() > 1) {
    void* d = be_->alloc(sizeof(unsigned long long) * K_);
    be_->copy(d, partial.data(), sizeof(unsigned long long) * K_, CopyKind::H2D, kReduce);
    comm_->allreduce(d, K_, RedType::U64, RedOp::Max, *be_, kReduce);
    be_->copy(partial.data(), d, sizeof(unsigned long long) * K_, CopyKind::D2H, kReduce);
    be_->sync(kReduce);
    be_->release(d);
  }
  long_major_ = partial[0] == 0;
  long_rem_ = 0;
  for (int r = 1; r < K_; ++r)
    if (!partial[r]) long_rem_ |= 1u << r;
  be_->sync_all();
}

double Solver::link_probe(std::size_t bytes, int reps) {
  if (comm_->all_local() || comm_->size() < 2 || bytes == 0) return 0.0;
  const int r = process_rank(), n = comm_->size();
  const int up = (r + 1) % n, dn = (r + n - 1) % n;
  const int npeer = up == dn ? 1 : 2;
  struct Bufs {  // released on every exit
    Backend* be;
    void *s = nullptr, *d = nullptr;
    ~Bufs() {
      be->release(s);
      be->release(d);
    }
  } b{be_.get(), be_->alloc(npeer * bytes), be_->alloc(npeer * bytes)};
  be_->memset(b.s, 0, npeer * bytes, kComm);
  std::vector<Transfer> xs;
  const int peers[2] = {up, dn};
  for (int i = 0; i < npeer; ++i) {
    Transfer snd, rcv;
    snd.src_rank = r;
    snd.dst_rank = peers[i];
    snd.src = static_cast<char*>(b.s) + i * bytes;
    snd.bytes = bytes;
    // the message from peer i arrives in slot i
    rcv.src_rank = peers[i];
    rcv.dst_rank = r;
    rcv.dst = static_cast<char*>(b.d) + i * bytes;
    rcv.bytes = bytes;
    xs.push_back(snd);
    xs.push_back(rcv);
  }
  be_->sync_all();
  double best = 1e30;
  for (int i = 0; i < 2 + std::max(1, reps); ++i) {
    comm_->barrier(*be_);
    const double t0 = now_s();
    comm_->exchange(xs, *be_, kComm);
    be_->sync(kComm);
    const double t = now_s() - t0;
    if (i >= 2) best = std::min(best, t);  // two warm-up exchanges (connection setup)
  }
  comm_->check_async_error();
  // the slowest rank decides: max over ranks of 2^62 - rate (in MB/s)
  const double mbps = (double)bytes / std::max(best, 1e-9) / 1e6;
  const unsigned long long big = 1ull << 62;
  unsigned long long v = big - (unsigned long long)std::max(0.0, std::min(mbps, 1e15));
  void* d = be_->alloc(8);
  be_->copy(d, &v, 8, CopyKind::H2D, kReduce);
  comm_->allreduce(d, 1, RedType::U64, RedOp::Max, *be_, kReduce);
  be_->copy(&v, d, 8, CopyKind::D2H, kReduce);
  be_->sync(kReduce);
  be_->release(d);
  return (double)(big - v) / 1e3;
}

int Solver::preheat(int sweeps) {
  if (!tb_ || sweeps <= 0) return 0;
  // Ordered behind every issued sweep and convergence check (join_pipeline),
  // the warm-up sweeps carry the device done flag without residual slots
  // (StencilParams::residual = false): once any issued iteration has met the
  // criterion they are no-ops, so nxt(cur()) — with two buffers the input of
  // the last sweep, which finalize_converged() needs for the rollback — is
  // only rewritten while no rollback can need it, and then with the values
  // the next sweep writes there anyway (a sweep is idempotent).
  join_pipeline();
  const int Kp = K_;
  int n = 0;
  for (int i = 0; i < sweeps; ++i) {
    for (auto& l : local_) {
      if (l.tb_interior.empty()) continue;
      StencilParams sp;
      sp.in = l.field[cur()];
      sp.out = l.field[nxt(cur())];
      sp.L = l.L;
      sp.box = l.tb_interior;
      for (int a = 0; a < 3; ++a) sp.D[a] = phys_.D[a];
      sp.state = dstate_;
      sp.residual = false;
      sp.cu_reserved = be_->reserved_cus();
      auto shrink = [&](const int64_t (&u)[2], int64_t nn, int64_t (&o)[2]) {
        o[0] = u[0] < 0 ? -(Kp - 1) : u[0];
        o[1] = u[1] > nn ? nn + Kp - 1 : u[1];
      };
      shrink(l.ux, l.sd.n[0], sp.ux);
      shrink(l.uy, l.sd.n[1], sp.uy);
      shrink(l.uz, l.sd.n[2], sp.uz);
      be_->sweep(dt_, sp, kspec2_, kCompute);
      ++n;
    }
  }
  // the next sweep's inputs and events are as they were; every stream orders
  // its later work behind the preheat (its output planes overlap the next
  // sweep's boundary slabs, which write the same values)
  ev_record(EV_FORK, kCompute);
  ev_wait(kComm, EV_FORK);
  ev_wait(kReduce, EV_FORK);
  return n;
}

// --- one iteration -----------------------------------------------------------
void Solver::enqueue_halo(int p, StreamId s, int dv) {
  // p = buffer index whose faces / ghosts are exchanged
  be_->range_push("halo");
  prof_record(prof_idx_, PE_HALO0, s);
  // one phase per axis when edges / corners must follow the faces
  // (ordered_halo_), else all faces at once
  const int nphase = ordered_halo_ ? 3 : 1;
  for (int ph = 0; ph < nphase; ++ph) {
    auto in_phase = [&](const FaceIO& io) { return !ordered_halo_ || face_axis(io.face) == ph; };
    enqueue_halo_phase(p, s, dv, in_phase);
  }
  prof_record(prof_idx_, PE_HALO1, s);
  be_->range_pop();
}

template <typename Pred>
void Solver::enqueue_halo_phase(int p, StreamId s, int dv, Pred in_phase) {
  if (comm_->all_local()) {
    for (auto& l : local_)
      for (auto& io : l.faces) {
        if (!in_phase(io)) continue;
        const Local& nb = local_[io.peer_local];
        const Box* src = nullptr;
        for (auto& nio : nb.faces)
          if (nio.face == opposite(io.face)) src = &nio.g[dv].send_box;
        HEAT3D_CHECK(src, "opposite face missing");
        be_->copy_box(dt_, nb.field[p], nb.L, *src, l.field[p], l.L, io.g[dv].recv_box, s);
      }
  } else {
    std::vector<Transfer> xs;
    for (auto& l : local_) {
      char* base = static_cast<char*>(l.field[p]);
      for (auto& io : l.faces) {
        if (!in_phase(io)) continue;
        const FaceGeom& fg = io.g[dv];
        if (!io.contiguous) be_->pack_box(dt_, l.field[p], l.L, fg.send_box, io.sendbuf, s);
        Transfer snd, rcv;
        snd.src_rank = l.sd.rank;
        snd.dst_rank = io.peer;
        snd.src = io.contiguous ? base + fg.send_off * esize_ : io.sendbuf;
        snd.bytes = fg.elems * esize_;
        rcv.src_rank = io.peer;
        rcv.dst_rank = l.sd.rank;
        rcv.dst = io.contiguous ? base + fg.recv_off * esize_ : io.recvbuf;
        rcv.bytes = fg.elems * esize_;
        xs.push_back(snd);
        xs.push_back(rcv);
      }
    }
    if (!xs.empty()) {
      comm_token_wait(s);
      prof_record(prof_idx_, PE_XCHG0, s);  // first phase: the transfer may start
      comm_->exchange(xs, *be_, s);
      comm_token_signal(s);
    }
    for (auto& l : local_)
      for (auto& io : l.faces)
        if (in_phase(io) && !io.contiguous) be_->unpack_box(dt_, l.field[p], l.L, io.g[dv].recv_box, io.recvbuf, s);
  }
}


void Solver::enqueue_iteration(int p, int bi) {
  H3D_TRACE("iteration issued=" << issued_ << " parity=" << p << " buf=" << bi
                                << (capturing_ ? " (capturing)" : ""));
  auto params = [&](Local& l, const Box& b) {
    StencilParams sp;
    sp.in = l.field[bi];
    sp.out = l.field[nxt(bi)];
    sp.L = l.L;
    sp.box = b;
    for (int a = 0; a < 3; ++a) sp.D[a] = phys_.D[a];
    sp.state = dstate_;
    sp.slot = p;
    return sp;
  };
  // per-phase timer events (diagnostic mode: one synchronised iteration at a time)
  auto T = [&](int i, StreamId s) {
    if (phase_timing_) be_->record(tev_[i], s);
  };
  if (last_kind_ != 1) join_pipeline();
  last_kind_ = 1;
  // [A] interior sweep on the compute stream
  ev_wait(kCompute, EV_CHK + p);  // convergence check of iteration t-2 (flag + slot reset)
  T(0, kCompute);
  if (overlap_) {
    ev_wait(kCompute, EV_BND + (p ^ 1));  // shell of t-1 written (and read) before we overwrite
    be_->range_push("interior");
    for (auto& l : local_) be_->stencil(dt_, params(l, l.interior), kspec_, kCompute);
    be_->range_pop();
    T(1, kCompute);
    ev_record(EV_INT + p, kCompute);
    // [B] halo exchange + shell on the comm stream
    ev_wait(kComm, EV_INT + (p ^ 1));  // interior of t-1 done (RAW on layer 1, WAR on shell)
    ev_wait(kComm, EV_CHK + p);
    T(2, kComm);
    enqueue_halo(bi, kComm);
    T(3, kComm);
    be_->range_push("shell");
    for (auto& l : local_)
      for (const Box& b : l.shell) be_->stencil(dt_, params(l, b), kspec_, kComm);
    be_->range_pop();
    T(4, kComm);
    ev_record(EV_BND + p, kComm);
  } else {
    T(2, kCompute);
    if (has_halo_) enqueue_halo(bi, kCompute);
    T(3, kCompute);
    be_->range_push("sweep");
    for (auto& l : local_) be_->stencil(dt_, params(l, l.owned), kspec_, kCompute);
    be_->range_pop();
    T(1, kCompute);
    T(4, kCompute);
    ev_record(EV_INT + p, kCompute);
  }
  // [C] global residual + convergence check on the reduce stream
  ev_wait(kReduce, EV_INT + p);
  if (overlap_) ev_wait(kReduce, EV_BND + p);
  T(5, kReduce);
  reduce_and_check(kReduce, p, 1);
  T(6, kReduce);
  ev_record(EV_CHK + p, kReduce);
}

// K iterations t..t+K-1 as one temporally blocked sweep: T^t in field[bi]
// -> T^{t+K} in field[bi^1], the K residuals fused (slots 0..K-1), then the K
// convergence checks.  The next sweep is queued behind those checks, so once
// converged it is a no-op and field[bi] (T^t with its halo) stays intact for
// the rollback in finalize_converged().
//
// Single subdomain: everything on the compute stream (graph-capturable).
// x slabs (pipeline events indexed by sweep parity q):
//   compute: wait check(q-L) + boundary(q-1) - interior planes [K, n0-K) - INT
//   comm   : K-plane halo of T^t - wait interior(q-1) + check(q-L) - boundary slabs - BND
//   reduce : wait INT, BND - allreduce(max) of the K residual slots - K checks - CHK
// The halo of sweep k+1 only depends on sweep k's boundary slabs, so it
// overlaps sweep k's interior tail and its all-reduce.  L = 1 with two
// buffers; with three (lag_) L = 2: the all-reduce and check of sweep q run
// under sweep q+1, whose residuals go to the other slot bank; if sweep q
// converged, q+1 was speculative (its output buffer is not q's input) and
// q+2 onwards are no-ops.  Exchanged values stay bitwise identical.
void Solver::enqueue_multi(int bi, int Kp, bool thick) {
  // Kp < K_: a partial sweep of Kp steps (the remainder of a step count that
  // is not a multiple of K_), same schedule and buffers, kernel of depth Kp;
  // Kp = K_ + 1: a long sweep (long_sweeps_for: single subdomain, or K+1-deep
  // ghosts with long_halo_), whose exchange and boundary layers are K+1 deep
  if (Kp <= 0) Kp = K_;
  HEAT3D_CHECK(Kp <= K_ || (Kp == K_ + 1 && (!has_halo_ || long_halo_)),
               "sweep depth " << Kp << " exceeds the halo depth " << K_);
  const int dv = Kp > K_ ? 1 : 0;
  // boundary pieces K+1 deep for long sweeps and for the sweep before one
  const bool lb = dv || (thick && long_halo_);
  H3D_TRACE("sweep" << Kp << " issued=" << issued_ << " buf=" << bi << (capturing_ ? " (capturing)" : ""));
  HEAT3D_CHECK(tb_, "temporal blocking not enabled for this decomposition");
  if (last_kind_ != 2) join_pipeline();
  last_kind_ = 2;
  // lagged schedule: events and residual slots alternate by sweep parity
  const int q = lag_ ? (int)(nsweep_ & 1) : bi;
  const int slot0 = lag_ ? q * slot_stride_ : 0;
  // partial (Kp < K) or long (Kp = K + 1) sweeps: the kernel family's default
  // variant of depth Kp, or the one the start-up timing kept
  const KernelSpec ks = spec_for_depth(Kp);
  // sweeps after iteration 0 (which sets the norm): the interior computes
  // only the last residual (residual_last_ok; boundary pieces compute all of
  // theirs, which the check ignores but the last); a converging sweep is
  // replayed by resolve_coarse
  const bool rl = Kp >= 2 && Kp < 8 && rl_d_[Kp] && issued_ > 0;
  const KernelSpec& kx = rl ? ks_last_[Kp] : ks;
  // update ranges reach Kp - 1 (not K_ - 1) points into the deep halos
  auto shrink = [&](const int64_t (&u)[2], int64_t n, int64_t (&o)[2]) {
    o[0] = u[0] < 0 ? -(Kp - 1) : u[0];
    o[1] = u[1] > n ? n + Kp - 1 : u[1];
  };
  auto params = [&](Local& l, const Box& b) {
    StencilParams sp;
    sp.in = l.field[bi];
    sp.out = l.field[nxt(bi)];
    sp.L = l.L;
    sp.box = b;
    for (int a = 0; a < 3; ++a) sp.D[a] = phys_.D[a];
    sp.state = dstate_;
    sp.slot = slot0;
    sp.cu_reserved = be_->reserved_cus();
    shrink(l.ux, l.sd.n[0], sp.ux);
    shrink(l.uy, l.sd.n[1], sp.uy);
    shrink(l.uz, l.sd.n[2], sp.uz);
    return sp;
  };
  if (!tb_overlap_) {
    ev_wait(kCompute, EV_CHK + 0);
    ev_wait(kCompute, EV_CHK + 1);
    if (has_halo_) enqueue_halo(bi, kCompute, dv);
    be_->range_push("sweep");
    prof_record(prof_idx_, PE_INT0, kCompute);
    // one subdomain, nothing to all-reduce: the sweep's last workgroup runs
    // the check (no check kernel and its dispatch on the critical path)
    const bool fused = fused_check();
    for (auto& l : local_) {
      StencilParams sp = params(l, dv ? l.tb_interior_long : l.tb_interior);
      sp.fuse_check = fused;
      be_->sweep(dt_, sp, kx, kCompute);
    }
    prof_record(prof_idx_, PE_INT1, kCompute);
    be_->range_pop();
    prof_record(prof_idx_, PE_RED0, kCompute);
    if (!fused) reduce_and_check(kCompute, slot0, Kp, prof_idx_, rl);
    prof_record(prof_idx_, PE_CHK1, kCompute);
    if (!capturing_) {
      for (int i = 0; i < 2; ++i) {
        ev_record(EV_INT + i, kCompute);
        ev_record(EV_BND + i, kCompute);
      }
    }
    ev_record(EV_CHK + 0, kCompute);
    ev_record(EV_CHK + 1, kCompute);
    return;
  }
  // Which check must precede this sweep's writes: it overwrites buffer
  // nxt(bi), the input of sweep q-1 (2 buffers) or q-2 (3 buffers), which a
  // convergence inside that sweep needs for the rollback; the same check
  // resets the residual slots this sweep writes.  EV_CHK + (q ^ 1) is sweep
  // q-1's check in both schedules' indexing; with the lag, EV_CHK + q still
  // stands for sweep q-2's (q's is recorded below).
  const int chk_prev = lag_ ? q : (q ^ 1);
  // [B1] the deep halo of T^t first in the collective chain: it depends only
  // on the previous sweep's boundary slabs (comm-stream order) and must not
  // queue behind the previous sweep's all-reduce, which waits for that
  // sweep's interior; the deferred all-reduce + check follow it.  Without the
  // lag this sweep's interior waits for that check (chk_prev), so it is issued
  // after the flush.
  // the halo sends the owned planes [0, d) / [n-d, n) of T^t, written by the
  // previous sweep's boundary slabs (comm-stream order) — unless they were
  // thinner than d, when the previous interior wrote the rest: wait for it
  // (a long sweep right after a K-thick one, e.g. across step() calls)
  if (last_bnd_ > 0 && (dv ? K_ + 1 : K_) > last_bnd_) ev_wait(kComm, EV_INT + (q ^ 1));
  last_bnd_ = lb ? K_ + 1 : K_;
  const StreamId sb = kComm;
  auto boundary_boxes = [&](Local& l) -> const std::vector<Box>& { return lb ? l.tb_boundary_long : l.tb_boundary; };
  // thin x-slab boundary pieces keep the y-marching thin-slab tiles whatever
  // tile shape --kernel2 gives the interior (the shape fields pick the form)
  auto bspec = [&](const Box& b) {
    if (b.extent(0) > Kp + 1) return ks;
    KernelSpec t = ks;
    t.V = t.R = t.WZ = t.WY = t.NT = t.L = t.ZS = 0;
    return t;
  };
  enqueue_halo(bi, kComm, dv);
  flush_pending_reduce();
  // [A] interior planes: they read the planes the previous sweep's boundary
  // slabs wrote.  (Round 4's core/rim split, a core that did not wait for
  // them plus thin rims that did, lost: each 3-plane rim took 46-77 us in
  // the thin-slab kernel, profiles/rank_proxy_r04.md.)
  ev_wait(kCompute, EV_CHK + chk_prev);
  be_->range_push("interior");
  prof_record(prof_idx_, PE_INT0, kCompute);
  ev_wait(kCompute, EV_BND + (q ^ 1));
  for (auto& l : local_) be_->sweep(dt_, params(l, lb ? l.tb_interior_long : l.tb_interior), kx, kCompute);
  prof_record(prof_idx_, PE_INT1, kCompute);
  be_->range_pop();
  ev_record(EV_INT + q, kCompute);
  // [B2] the boundary slabs, behind the halo on the comm stream.  (Round 4's
  // opt-in alternative, the boundary pieces after the interior on the
  // compute stream, was removed in round 5: config 5's share ran 6.97
  // against 6.65 ms/step with it, the 8-GPU slab share 0.231 against 0.209;
  // profiles/r05/proxy_runs.md.)
  ev_wait(kComm, EV_INT + (q ^ 1));  // previous interior read the planes we overwrite
  ev_wait(kComm, EV_CHK + chk_prev);
  be_->range_push("boundary");
  prof_record(prof_idx_, PE_BND0, sb);
  for (auto& l : local_)
    for (const Box& b : boundary_boxes(l)) be_->sweep(dt_, params(l, b), bspec(b), sb);
  prof_record(prof_idx_, PE_BND1, sb);
  be_->range_pop();
  ev_record(EV_BND + q, sb);
  // [C] all residuals, all checks: now, or (ordered collectives) after the
  // next sweep's halo.  With the lag nothing waits for CHK(q) before sweep
  // q+2; without it sweep q+1's interior does, and is issued after the flush.
  pending_.valid = true;
  pending_.q = q;
  pending_.slot0 = slot0;
  pending_.Kp = Kp;
  pending_.prof = prof_idx_;
  pending_.last_only = rl;
  if (!chain_) flush_pending_reduce();
  ++nsweep_;
}

bool Solver::fused_check() const {
  return cfg_.fuse_check && be_->is_gpu() && tb_ && !tb_overlap_ && local_.size() == 1 &&
         (comm_->all_local() || comm_->size() == 1) && fake_allreduce_us_ <= 0;
}

// Monotone check.  With c = 1 - 2(Dx + Dy + Dz) >= 0 the update is a convex
// combination, T'_p = c T_p + sum_a D_a (T_{p-a} + T_{p+a}), and so is the
// change it makes: T''_p - T'_p is the same combination of the changes T' - T
// at p and its neighbours, which are 0 on the fixed boundary.  Hence
// max|T'' - T'| <= max|T' - T|: the residual never grows, and a sweep whose
// last residual is at or above the threshold has no converged step.  (In
// floating point the residuals are those of the rounded fields; the rounding
// moves them by ~1e-16 of the field, against a threshold-crossing step of
// ~1e-10 of it at 1024^3, eps 1e-5.)  Converged sweeps are replayed with all
// residuals (resolve_coarse), so conv_iter, last_residual and the fields are
// those of the every-step check.  With more than one rank the replay
// all-reduces its residuals: state() is then collective once a run has
// converged in such a sweep (run() calls it on every rank).
bool Solver::residual_last_ok() const {
  const double c = 1.0 - 2.0 * (phys_.D[0] + phys_.D[1] + phys_.D[2]);
  return cfg_.monotone_check && be_->is_gpu() && tb_ && cfg_.verbose <= 0 && c >= 0.0 && fake_allreduce_us_ <= 0;
}

KernelSpec Solver::last_only(const KernelSpec& ks) const {
  KernelSpec r = ks.resolved(dt_);
  r.O = (r.O > 0 ? r.O : 0) | kResidualLastOnly;
  return r;
}

void Solver::resolve_coarse() {
  DeviceState& h = *hstate_;  // state(): a fresh copy of the device state
  const int64_t c = h.conv_iter;
  const int kc = (int)h.coarse;
  const Segment* hit = nullptr;
  for (const auto& sg : segs_)
    if (c >= sg.start && c < sg.start + sg.len) hit = &sg;
  HEAT3D_CHECK(hit && hit->len == kc && c == hit->start + kc - 1 && kc <= kResidualSlots,
               "monotone check: sweep of iteration " << c << " (" << kc << " steps) not recorded");
  if (!rstate_) rstate_ = static_cast<DeviceState*>(be_->alloc(sizeof(DeviceState)));
  // scratch state: only the residual slots and the done flag are read
  DeviceState z;
  std::memset(&z, 0, sizeof(z));
  for (auto& r : z.residual) r = kResidualInitBits;
  be_->copy(rstate_, &z, offsetof(DeviceState, hist), CopyKind::H2D, kCompute);
  // every piece of the sweep (interior, and the boundary slabs of overlapped
  // schedules) from its input buffer, which still holds T^start and its deep
  // halo (as finalize_converged relies on); the interior in the sweep's shape,
  // the boundary pieces in the kernel family's default variant of its depth
  // (every variant computes the same bits)
  KernelSpec kd;
  kd.kind = kspec2_.kind;
  kd.K = kc;
  const bool lng = kc > K_;
  for (auto& l : local_) {
    std::vector<Box> pieces{lng ? l.tb_interior_long : l.tb_interior};
    if (tb_overlap_) {
      const std::vector<Box>& bnd = lng ? l.tb_boundary_long : l.tb_boundary;
      pieces.insert(pieces.end(), bnd.begin(), bnd.end());
    }
    for (std::size_t i = 0; i < pieces.size(); ++i) {
      const Box& b = pieces[i];
      if (b.empty()) continue;
      StencilParams sp;
      sp.in = l.field[hit->inbuf];
      sp.out = l.field[nxt(hit->inbuf)];  // rewritten with the values it holds
      sp.L = l.L;
      sp.box = b;
      for (int a = 0; a < 3; ++a) sp.D[a] = phys_.D[a];
      sp.state = rstate_;
      sp.slot = 0;
      sp.cu_reserved = be_->reserved_cus();
      auto shrink = [&](const int64_t (&u)[2], int64_t n, int64_t (&o)[2]) {
        o[0] = u[0] < 0 ? -(kc - 1) : u[0];
        o[1] = u[1] > n ? n + kc - 1 : u[1];
      };
      shrink(l.ux, l.sd.n[0], sp.ux);
      shrink(l.uy, l.sd.n[1], sp.uy);
      shrink(l.uz, l.sd.n[2], sp.uz);
      be_->sweep(dt_, sp, i == 0 ? spec_for_depth(kc) : kd, kCompute);
    }
  }
  if (!comm_->all_local() && comm_->size() > 1) {
    comm_token_wait(kCompute);
    comm_->allreduce(rstate_->residual, kc, RedType::U64, RedOp::Max, *be_, kCompute);
    comm_token_signal(kCompute);
  }
  unsigned long long bits[kResidualSlots];
  be_->copy(bits, rstate_->residual, sizeof(unsigned long long) * kc, CopyKind::D2H, kCompute);
  be_->sync(kCompute);
  bool found = false;
  for (int j = 0; j < kc && !found; ++j) {
    const double r = __builtin_bit_cast(double, bits[j]);
    const int64_t t = hit->start + j;
    if (!(r == r) || r > 1.7976931348623157e308) {  // as check_convergence_scalar
      h.fault = 1;
      found = true;
    } else if (r / h.norm < h.eps) {
      found = true;
    }
    if (found) {
      h.conv_iter = t;
      h.last_residual = r;
    }
  }
  HEAT3D_CHECK(found, "monotone check: the replayed sweep of iterations " << hit->start << ".." << c
                                                                          << " has no converged step");
  H3D_TRACE("monotone check: sweep " << hit->start << ".." << c << " converged at " << h.conv_iter);
  h.coarse = 0;
  // the resolved fields back to the device state (done stays set)
  char* d = reinterpret_cast<char*>(dstate_);
  be_->copy(d + offsetof(DeviceState, last_residual), &h.last_residual, sizeof(double), CopyKind::H2D, kCompute);
  be_->copy(d + offsetof(DeviceState, conv_iter), &h.conv_iter, sizeof(int64_t), CopyKind::H2D, kCompute);
  be_->copy(d + offsetof(DeviceState, fault), &h.fault, sizeof(int32_t), CopyKind::H2D, kCompute);
  be_->copy(d + offsetof(DeviceState, coarse), &h.coarse, sizeof(uint32_t), CopyKind::H2D, kCompute);
  be_->sync(kCompute);
}

void Solver::reduce_and_check(StreamId s, int slot0, int Kp, int prof, bool last_only) {
  if (!comm_->all_local() && comm_->size() > 1) {
    comm_token_wait(s);
    comm_->allreduce(&dstate_->residual[slot0], Kp, RedType::U64, RedOp::Max, *be_, s);
    comm_token_signal(s);
  } else if (fake_allreduce_us_ > 0) {
    be_->delay(fake_allreduce_us_, s);  // single-GPU stand-in for the RCCL latency
  }
  prof_record(prof, PE_REDX, s);
  be_->check_convergence(dstate_, slot0, s, Kp, last_only);
}

void Solver::flush_pending_reduce() {
  if (!pending_.valid) return;
  pending_.valid = false;
  const int q = pending_.q;
  const StreamId sr = kReduce;
  ev_wait(sr, EV_INT + q);
  ev_wait(sr, EV_BND + q);
  prof_record(pending_.prof, PE_RED0, sr);
  reduce_and_check(sr, pending_.slot0, pending_.Kp, pending_.prof, pending_.last_only);
  prof_record(pending_.prof, PE_CHK1, sr);
  ev_record(EV_CHK + q, sr);
}

void Solver::prof_record(int sweep, int id, StreamId s) {
  if (!prof_on_ || sweep < 0 || capturing_) return;
  unsigned& set = prof_set_[sweep];
  if (set & (1u << id)) return;  // first occurrence only (e.g. the first halo phase)
  set |= 1u << id;
  be_->record(prof_ev_[(std::size_t)sweep * PE_COUNT + id], s);
}

std::vector<std::pair<std::string, double>> Solver::profile_sweeps(int n) {
  std::vector<std::pair<std::string, double>> out;
  if (!tb_ || n < 3) return out;
  flush_pending_reduce();
  const std::size_t need = (std::size_t)n * PE_COUNT;
  while (prof_ev_.size() < need) prof_ev_.push_back(be_->event_create());
  prof_set_.assign(n, 0u);
  prof_on_ = true;
  try {
    for (int i = 0; i < n; ++i) {
      prof_idx_ = i;
      record_segment(issued_, K_, cur());
      enqueue_multi(cur(), K_);
      issued_ += K_;
      cur_ = nxt(cur_);
    }
    prof_idx_ = -1;
    flush_pending_reduce();
    be_->sync_all();
  } catch (...) {
    prof_on_ = false;
    prof_idx_ = -1;
    throw;
  }
  prof_on_ = false;
  comm_->check_async_error();
  auto ev = [&](int i, int id) { return prof_ev_[(std::size_t)i * PE_COUNT + id]; };
  auto has = [&](int i, int id) { return (prof_set_[i] >> id) & 1u; };
  auto ms = [&](int i, int a, int j, int b) { return (double)be_->elapsed_ms(ev(i, a), ev(j, b)); };
  // sweeps 1 .. n-2: every one has a predecessor and a successor in the window
  std::map<std::string, std::pair<double, int>> acc;
  auto add = [&](const char* k, double v) {
    auto& a = acc[k];
    a.first += v;
    a.second += 1;
  };
  for (int i = 1; i + 1 < n; ++i) {
    if (!has(i, PE_INT0) || !has(i, PE_INT1)) continue;
    add("interior_ms", ms(i, PE_INT0, i, PE_INT1));
    add("sweep_ms", ms(i, PE_INT0, i + 1, PE_INT0));
    add("compute_idle_ms", ms(i, PE_INT1, i + 1, PE_INT0));
    if (has(i, PE_HALO0) && has(i, PE_HALO1)) {
      add("halo_ms", ms(i, PE_HALO0, i, PE_HALO1));
      if (has(i, PE_XCHG0)) {
        add("halo_token_wait_ms", ms(i, PE_HALO0, i, PE_XCHG0));
        add("halo_transfer_ms", ms(i, PE_XCHG0, i, PE_HALO1));
      }
    }
    if (has(i, PE_BND0) && has(i, PE_BND1)) {
      add("boundary_ms", ms(i, PE_BND0, i, PE_BND1));
      if (has(i, PE_HALO1)) add("boundary_wait_ms", ms(i, PE_HALO1, i, PE_BND0));
      // boundary chain end relative to the interior's end (> 0: exposed tail)
      add("boundary_tail_ms", ms(i, PE_INT1, i, PE_BND1));
      if (has(i, PE_HALO0)) {
        // overlap of [halo start, boundary end] with [interior start, end]
        const double c0 = ms(i, PE_INT0, i, PE_HALO0), c1 = ms(i, PE_INT0, i, PE_BND1);
        const double e = ms(i, PE_INT0, i, PE_INT1);
        const double lo = std::max(0.0, c0), hi = std::min(e, c1);
        add("chain_overlap_fraction", c1 > c0 ? std::max(0.0, hi - lo) / (c1 - c0) : 0.0);
        add("halo_start_after_interior_start_ms", c0);
      }
    }
    if (has(i, PE_RED0) && has(i, PE_REDX) && has(i, PE_CHK1)) {
      add("allreduce_ms", ms(i, PE_RED0, i, PE_REDX));
      add("check_ms", ms(i, PE_REDX, i, PE_CHK1));
    }
  }
  out.push_back({"sweeps", (double)(n - 2)});
  out.push_back({"steps_per_sweep", (double)K_});
  for (auto& kv : acc) out.push_back({kv.first, kv.second.first / std::max(1, kv.second.second)});
  return out;
}

void Solver::comm_token_wait(StreamId s) {
  if (chain_) ev_wait(s, EV_TOKEN);
}

void Solver::comm_token_signal(StreamId s) {
  if (chain_) ev_record(EV_TOKEN, s);
}

void Solver::join_pipeline() {
  flush_pending_reduce();
  for (StreamId s : {kCompute, kComm, kReduce}) {
    for (int id = EV_INT; id < EV_CHK + 2; ++id) ev_wait(s, id);
    ev_wait(s, EV_TOKEN);
  }
}

void Solver::record_segment(int64_t start, int len, int inbuf) {
  const std::size_t cap = 1 << 14;
  if (segs_.size() < cap) segs_.push_back({start, len, inbuf});
  else segs_[seg_head_ % cap] = {start, len, inbuf};
  ++seg_head_;
}

// After convergence at iteration c the final field is T^{c+1}.  Find the
// segment that computed iteration c; a temporally blocked pair that met the
// criterion in its first half stored T^{c+2}, so recompute T^{c+1} from its
// (untouched) input buffer with one forced single step.
void Solver::finalize_converged(int64_t c) {
  be_->sync_all();
  const Segment* hit = nullptr;
  for (const auto& s : segs_)
    if (c >= s.start && c < s.start + s.len) hit = &s;
  HEAT3D_CHECK(hit, "segment of converged iteration " << c << " not recorded");
  const Segment s = *hit;
  const int m = (int)(c - s.start + 1);  // steps of the segment that are wanted
  int final_buf = nxt(s.inbuf);
  if (m < s.len) {
    // The sweep's input buffer still holds T^start with its K-deep halo (the
    // later, no-op sweeps only re-exchanged unchanged faces into it).  Redo
    // m forced single steps; step j also updates m-j halo planes on faces
    // with a neighbour, so no exchange is needed in between.
    for (int j = 1; j <= m; ++j) {
      const int src = (j & 1) ? s.inbuf : nxt(s.inbuf);
      const int dst = (j & 1) ? nxt(s.inbuf) : s.inbuf;
      for (auto& l : local_) {
        StencilParams sp;
        sp.in = l.field[src];
        sp.out = l.field[dst];
        sp.L = l.L;
        sp.box = l.owned;
        const int64_t w = m - j;
        for (int a = 0; a < 3; ++a) {
          if (hd_[a] <= 1) continue;
          if (l.sd.has_neighbor(static_cast<Face>(2 * a))) sp.box.lo[a] -= w;
          if (l.sd.has_neighbor(static_cast<Face>(2 * a + 1))) sp.box.hi[a] += w;
        }
        for (int a = 0; a < 3; ++a) sp.D[a] = phys_.D[a];
        sp.state = nullptr;  // forced: ignores the done flag, no residual
        be_->stencil(dt_, sp, kspec_, kCompute);
      }
    }
    be_->sync(kCompute);
    final_buf = (m & 1) ? nxt(s.inbuf) : s.inbuf;
  }
  issued_ = c + 1;
  cur_ = final_buf;
}

void Solver::accumulate_phase_times() {
  be_->sync_all();
  static const char* names[] = {"interior_ms", "halo_ms", "shell_ms", "reduce_check_ms", "iteration_ms"};
  const double v[5] = {be_->elapsed_ms(tev_[0], tev_[1]), be_->elapsed_ms(tev_[2], tev_[3]),
                       be_->elapsed_ms(tev_[3], tev_[4]), be_->elapsed_ms(tev_[5], tev_[6]),
                       be_->elapsed_ms(tev_[0], tev_[6])};
  if (phase_acc_.empty())
    for (auto* n : names) phase_acc_.push_back({n, 0.0});
  for (int i = 0; i < 5; ++i) phase_acc_[i].second += v[i];
  ++phase_count_;
}

// Iterations per captured graph for a chunk of n: --graph-chunk, or the
// largest whole number of schedule cycles <= n, so that a short run (the
// driver's 20-step bench) replays a graph too.  A cycle brings every rotating
// role back to its start: the buffer ring (2, or 3 with the lagged check), the
// event / residual-slot parity of single steps (2) and of overlapped sweeps (2).
int Solver::graph_len_for(int64_t n) const {
  int cyc;
  if (tb_) cyc = K_ * (nbuf_ == 3 ? 6 : 2);
  else cyc = nbuf_ == 3 ? 6 : 2;
  // auto: 32 iterations, 96 for the overlapped multi-stream schedule, whose
  // per-stream graphs start and end joined (each launch drains the halo /
  // boundary / all-reduce pipeline once: ~0.12 ms on the 8-GPU slab share,
  // 3% of 32-iteration chunks; profiles/graph_streams_r05.md)
  const int chunk = cfg_.graph_chunk > 0 ? cfg_.graph_chunk : multi_stream() ? 96 : 32;
  int G = std::max(cyc, chunk - chunk % cyc);
  if (n < G) G = (int)(n - n % cyc);
  // a step count shorter than one cycle (the driver's 20-step window at 8
  // ranks: 12 steps in K = 3 sweeps + 2 long sweeps; the 3-buffer cycle is
  // 18) is one graph too, replayable only from the same state
  if (G == 0 && tb_) G = (int)(n - n % K_);
  return G;
}

int Solver::long_sweeps_for(int64_t n) const {
  if (!tb_ || (has_halo_ && !long_halo_) || !kspec2_.multi_step()) return 0;
  if (K_ + 1 > 6 || K_ + 1 > kResidualSlots) return 0;
  if (long_major_ && cfg_.long_sweeps) {
    // the most long sweeps b with n - b (K + 1) a multiple of K (b = n mod K
    // modulo K); none fits: the remainder policy below
    const int64_t bmax = n / (K_ + 1), r = n % K_;
    const int64_t b = bmax - (((bmax - r) % K_) + K_) % K_;
    if (b > 0 && b * (K_ + 1) <= n && (n - b * (K_ + 1)) % K_ == 0) return (int)std::min<int64_t>(b, INT32_MAX);
  }
  if (n % K_ == 0) return 0;
  const int64_t b = n % K_;             // n = a K + b (K + 1) with a = (n - b (K + 1)) / K
  if (b * (K_ + 1) > n) return 0;
  if (!cfg_.long_sweeps || !((long_rem_ >> b) & 1u)) return 0;
  // the K+1 variant must exist for this dtype (e.g. fp64 K = 5 has no K = 6)
  KernelSpec ks;
  ks.kind = kspec2_.kind;
  ks.K = K_ + 1;
  return be_->is_gpu() && !hip::lean_supported(dt_, ks) ? 0 : (int)b;
}

bool Solver::graphs_allowed() const {
  // Multi-stream (overlapped) schedules replay one linear graph per stream,
  // each on its own stream with its CU mask and priority, the cross-stream
  // dependencies as device-side signal / wait kernels (HipBackend,
  // Backend::begin_capture).  (One fork/join DAG, the round-2..4 form, was
  // replayed by the HIP runtime on streams of its own without either: 0.366
  // against 0.212 ms/step eager on the 8-GPU slab share, profiles/rank_proxy_r04.md.)
  return cfg_.use_graph && be_->supports_graphs() && comm_->capturable() && !graph_failed_ && !phase_timing_ &&
         !force_eager_ && (!multi_stream() || stream_graphs_enabled());
}

// --stream-graphs auto replays the overlapped multi-stream schedule eagerly:
// on the 8-GPU slab share (phantom rank, driver window) eager ran 0.2233 /
// 0.2240 ms/step against 0.2314 / 0.2308 with the per-stream graphs (each
// launch joins and re-forks the streams, which drains the halo pipeline once:
// ~0.12 ms per launch; gpurun_out/r6p), and over 300 steps 0.2086 against
// 0.2115 (round 5) — the graphs' cheaper cross-stream waits (13 / 10 us per
// sweep against 31 / 41, profiles/r06/chain_gaps_8gpu_share.md) do not pay
// for it — and their device-side waits are a liveness hazard where queues are
// shared.  "on" records them (canary-verified), unless more than 4 processes
// share the GPU (the 8-rank one-GPU rehearsal oversubscribes its hardware
// queues: round 5's hang, round 6's canary deadlock).
bool Solver::stream_graphs_enabled() const {
  if (sg_fallback_ || cfg_.stream_graphs != 1) return false;
  return true;
}

Solver::GraphEntry* Solver::find_graph(int G, int kind_req) {
  const int kind = kind_req ? kind_req : tb_ ? 2 : 1;
  for (auto& g : graphs_)
    if (g.exec && g.G == G && g.kind == kind && g.buf == cur() && g.parity == (int)(issued_ & 1) &&
        g.sparity == (int)(nsweep_ & 1) && g.first == (issued_ == 0))
      return &g;
  return nullptr;
}

void Solver::destroy_graphs() {
  if (graphs_.empty()) return;
  be_->sync_all();
  for (auto& g : graphs_) be_->destroy_graph(g.exec);
  graphs_.clear();
}

// Capture G iterations, as run_chunk would issue them eagerly from the current
// state (fresh events for every record inside the capture): single-stream
// schedules into one graph on the compute stream, whose comm / reduce
// branches fork from it and join back into it; multi-stream schedules into
// one linear graph per stream (the backend forks and joins the streams around
// their launch).  The solver's host-side schedule state is restored
// afterwards: a launch advances it exactly like the eager path.
Solver::GraphEntry* Solver::build_graph(int G, int kind_req) {
  H3D_TRACE("build_graph G=" << G << " kind " << kind_req << " at issued=" << issued_);
  join_pipeline();
  GraphEntry e;
  e.G = G;
  e.kind = kind_req ? kind_req : tb_ ? 2 : 1;  // 3: K+1-step sweeps (long-major)
  e.buf = cur();
  e.parity = (int)(issued_ & 1);
  e.sparity = (int)(nsweep_ & 1);
  e.first = issued_ == 0;
  bool saved[EV_COUNT];
  std::memcpy(saved, ev_valid_, sizeof(saved));
  Event saved_cur[EV_COUNT];
  std::memcpy(saved_cur, cur_ev_, sizeof(saved_cur));
  const int64_t s_issued = issued_, s_nsweep = nsweep_;
  const int s_cur = cur_, s_last = last_kind_, s_bnd = last_bnd_;
  const std::size_t need = 16 * (std::size_t)G + 16;
  while (cap_pool_.size() < need) cap_pool_.push_back(be_->event_create());
  cap_next_ = 0;
  arm_segv_trace();
  const bool split = multi_stream();
  try {
    be_->begin_capture(split, dstate_, (int)need);
    capturing_ = true;
    for (int i = 0; i < EV_COUNT; ++i) ev_valid_[i] = false;
    if (!split) {
      ev_record(EV_FORK, kCompute);
      ev_wait(kComm, EV_FORK);
      ev_wait(kReduce, EV_FORK);
    }
    last_kind_ = e.kind == 3 ? 2 : e.kind;
    if (e.kind == 2) {
      for (int i = 0; i < G / K_; ++i) {
        enqueue_multi(cur_);
        issued_ += K_;
        cur_ = nxt(cur_);
      }
    } else if (e.kind == 3) {
      for (int i = 0; i < G / (K_ + 1); ++i) {
        enqueue_multi(cur_, K_ + 1);
        issued_ += K_ + 1;
        cur_ = nxt(cur_);
      }
    } else {
      for (int i = 0; i < G; ++i) {
        enqueue_iteration((int)(issued_ & 1), cur_);
        ++issued_;
        cur_ = nxt(cur_);
      }
    }
    flush_pending_reduce();
    if (!split) {
      ev_record(EV_JCOMM, kComm);
      ev_record(EV_JRED, kReduce);
      ev_wait(kCompute, EV_JCOMM);
      ev_wait(kCompute, EV_JRED);
    }
    H3D_TRACE("end_capture");
    capturing_ = false;
    e.exec = be_->end_capture();
    H3D_TRACE("graph instantiated");
  } catch (const std::exception& ex) {
    if (capturing_) {
      capturing_ = false;
      try {
        be_->destroy_graph(be_->end_capture());
      } catch (...) {
      }
    }
    e.exec = nullptr;
    graph_failed_ = true;
    if (!cfg_.quiet && is_root())
      std::fprintf(stderr, "heat3d: hipGraph capture failed (%s); running eagerly\n", ex.what());
  }
  issued_ = s_issued;
  nsweep_ = s_nsweep;
  cur_ = s_cur;
  last_kind_ = s_last;
  last_bnd_ = s_bnd;
  pending_.valid = false;
  std::memcpy(ev_valid_, saved, sizeof(saved));
  std::memcpy(cur_ev_, saved_cur, sizeof(saved_cur));
  if (!e.exec) return nullptr;
  if (graphs_.size() >= 8) {
    be_->sync_all();
    be_->destroy_graph(graphs_.front().exec);
    graphs_.erase(graphs_.begin());
  }
  graphs_.push_back(e);
  return &graphs_.back();
}

void Solver::prepare_steps(int64_t n) {
  if (!graphs_allowed()) return;
  const int nlong = long_sweeps_for(n);
  const int G = graph_len_for(n - (int64_t)nlong * (K_ + 1));
  if (G > 0 && !find_graph(G)) build_graph(G);
  // long-major: the first graph of long sweeps (run_chunk issues them after
  // the K-step part, whose graph ends on the same buffer it started from)
  const int m = std::min(nlong, long_graph_cap());
  if (long_major_ && !multi_stream() && m > 0 && G % (2 * K_) == 0 && !find_graph(m * (K_ + 1), 3))
    build_graph(m * (K_ + 1), 3);
}

// long-major graphs: at most this many K+1-step sweeps each (the graph chunk)
int Solver::long_graph_cap() const {
  const int chunk = cfg_.graph_chunk > 0 ? cfg_.graph_chunk : 32;
  return std::max(1, chunk / (K_ + 1));
}

void Solver::run_chunk(int64_t n) {
  const bool graphs = graphs_allowed();
  // remainder as long sweeps, issued after the graph-sized part
  const int nlong = long_sweeps_for(n);
  n -= (int64_t)nlong * (K_ + 1);
  while (n > 0) {
    const int G = graphs ? graph_len_for(n) : 0;
    if (G > 0) {
      GraphEntry* g = find_graph(G);
      if (!g) g = build_graph(G);
      if (g) {
        H3D_TRACE("launch_graph G=" << G << " issued=" << issued_);
        // the graph is launched on the compute stream: order it after work
        // still pending on the other streams (e.g. an overlapped single step)
        join_pipeline();
        be_->launch_graph(g->exec);
        ++graph_launches_;
        if (multi_stream()) sg_unchecked_ = true;
        if (g->kind == 2) {
          for (int i = 0; i < G / K_; ++i) {
            record_segment(issued_, K_, cur());
            issued_ += K_;
            cur_ = nxt(cur_);
            if (tb_overlap_) ++nsweep_;  // as enqueue_multi counts them
          }
        } else {
          for (int i = 0; i < G; ++i) {
            record_segment(issued_, 1, cur());
            ++issued_;
            cur_ = nxt(cur_);
          }
        }
        n -= G;
        last_kind_ = g->kind;
        last_bnd_ = 0;  // the graph ends joined into the compute stream (re-fork below)
        // the graph joined every stream into compute: re-fork for eager work
        for (int i = 0; i < EV_COUNT; ++i) ev_valid_[i] = false;
        ev_record(EV_FORK, kCompute);
        ev_wait(kComm, EV_FORK);
        ev_wait(kReduce, EV_FORK);
        continue;
      }
    }
    if (tb_ && n >= 2 && !phase_timing_) {
      // a full sweep, or a partial one for a remainder of 2 .. K-1 steps
      const int Kp = (int)std::min<int64_t>(n, K_);
      record_segment(issued_, Kp, cur());
      enqueue_multi(cur(), Kp, nlong > 0 && n == Kp);
      issued_ += Kp;
      cur_ = nxt(cur_);
      n -= Kp;
      continue;
    }
    if (phase_timing_ && !tev_[0])
      for (auto& e : tev_) e = be_->event_create();
    record_segment(issued_, 1, cur());
    enqueue_iteration((int)(issued_ & 1), cur());
    if (phase_timing_) accumulate_phase_times();
    ++issued_;
    cur_ = nxt(cur_);
    --n;
  }
  // long sweeps: long-major runs replay graphs of up to long_graph_cap() of
  // them (single-stream schedules), else eagerly
  int left = nlong;
  while (graphs && long_major_ && !multi_stream() && left > 0) {
    const int m = std::min(left, long_graph_cap());
    GraphEntry* g = find_graph(m * (K_ + 1), 3);
    if (!g) g = build_graph(m * (K_ + 1), 3);
    if (!g) break;
    H3D_TRACE("launch_graph long x" << m << " issued=" << issued_);
    join_pipeline();
    be_->launch_graph(g->exec);
    ++graph_launches_;
    for (int i = 0; i < m; ++i) {
      record_segment(issued_, K_ + 1, cur());
      issued_ += K_ + 1;
      cur_ = nxt(cur_);
    }
    left -= m;
    last_kind_ = 2;
    last_bnd_ = 0;
    for (int i = 0; i < EV_COUNT; ++i) ev_valid_[i] = false;
    ev_record(EV_FORK, kCompute);
    ev_wait(kComm, EV_FORK);
    ev_wait(kReduce, EV_FORK);
  }
  for (int i = 0; i < left; ++i) {
    record_segment(issued_, K_ + 1, cur());
    enqueue_multi(cur(), K_ + 1);
    issued_ += K_ + 1;
    cur_ = nxt(cur_);
  }
  flush_pending_reduce();
}

void Solver::step(int64_t n) { run_chunk(n); }

void Solver::synchronize() {
  be_->sync_all();
  comm_->check_async_error();
  check_graph_fault();
}

HostState Solver::state() {
  be_->sync_all();
  be_->copy(hstate_, dstate_, sizeof(DeviceState), CopyKind::D2H, kCompute);
  be_->sync(kCompute);
  if (hstate_->done && hstate_->coarse) resolve_coarse();
  HostState h;
  h.norm = hstate_->norm;
  h.eps = hstate_->eps;
  h.last_residual = hstate_->last_residual;
  h.error_sum = hstate_->error_sum;
  h.error_count = hstate_->error_count;
  h.iter = hstate_->iter;
  h.conv_iter = hstate_->conv_iter;
  h.done = hstate_->done;
  h.fault = hstate_->fault;
  return h;
}

RunResult Solver::run() {
  RunResult R;
  comm_->barrier(*be_);
  be_->sync_all();
  const double t0 = now_s();
  // poll chunks hold whole schedule cycles (graph_len_for), so that
  // temporally blocked runs stay aligned with their graphs and never fall
  // back to single steps; with graphs at least one whole graph, whose launch
  // joins the streams (the overlapped schedule drains its pipeline there)
  int64_t K = std::max(1, cfg_.check_every);
  if (tb_) {
    // long-major: chunks of whole K+1-step sweeps too (24 = 6 x 4)
    const int64_t cyc = (int64_t)K_ * (nbuf_ == 3 ? 6 : 2) * (long_major_ ? K_ + 1 : 1);
    if (graphs_allowed()) K = std::max<int64_t>(K, graph_len_for(INT32_MAX));
    K = std::max(cyc, K - K % cyc);
  }
  const std::size_t poll_bytes = cfg_.verbose > 0 ? sizeof(DeviceState) : offsetof(DeviceState, hist);
  int pslot = 0;
  bool have_prev = false, stop = false;
  int64_t next_ckpt = cfg_.checkpoint_every > 0 ? issued_ + cfg_.checkpoint_every : -1;
  int64_t next_verify = cfg_.verify_halo > 0 ? issued_ + cfg_.verify_halo : -1;
  if (cfg_.timers) set_phase_timing(true);
  int64_t printed = issued_;
  const int64_t iter0 = issued_;
  double last_beat = t0;
  int64_t iter_cap = cfg_.iter_max;        // --time-limit lowers it
  int64_t chunk_idx = 0, next_vote = 4;    // polled chunks; chunk of the next --time-limit vote
  const double watchdog = cfg_.watchdog_s;
  while (issued_ < iter_cap && !stop) {
    int64_t n = std::min(K, iter_cap - issued_);
    if (next_ckpt > 0) n = std::min(n, next_ckpt - issued_);
    run_chunk(n);
    // pinned copy of the device convergence state, polled one chunk later
    ev_wait(kReduce, EV_CHK + 0);
    ev_wait(kReduce, EV_CHK + 1);
    be_->copy(&hstate_[pslot], dstate_, poll_bytes, CopyKind::D2H, kReduce);
    ev_record(EV_POLL + pslot, kReduce);
    if (have_prev) {
      const int q = pslot ^ 1;
      const double tw = now_s();
      while (!be_->query(cur_ev_[EV_POLL + q])) {
        comm_->check_async_error();
        if (now_s() - tw > watchdog) {
          comm_->abort();
          HEAT3D_THROW("watchdog: no progress for " << watchdog << " s (peer failure?)");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
      const DeviceState& hs = hstate_[q];
      if (cfg_.verbose > 0 && is_root()) {
        for (int64_t it = printed; it < hs.iter; ++it)
          if (it % cfg_.verbose == 0 && it >= hs.iter - hs.hist_cap)
            std::printf("iteration %lld residual %.6e\n", (long long)it, hs.hist[it % hs.hist_cap]);
        printed = hs.iter;
      }
      if (hs.done) stop = true;
      // wall budget (--time-limit): an iteration cap voted at the same chunk
      // on every rank (a per-rank clock test could stop the ranks at
      // different chunks, and the collectives would no longer pair up):
      // each rank projects the iterations that fit from its completed rate,
      // the job takes the smallest (one all-reduce, in the collective order).
      // First after 4 chunks, then again every 8, so that a rate that drops
      // later (clocks, contention) lowers the cap again.
      ++chunk_idx;
      if (cfg_.time_limit_s > 0 && chunk_idx >= next_vote) {
        next_vote = chunk_idx + 8;
        const double el = now_s() - t0;
        const double rate = el > 0 ? (double)(hs.iter - iter0) / el : 0.0;
        int64_t cap = hs.iter + (int64_t)(rate * std::max(0.0, cfg_.time_limit_s - el));
        if (!comm_->all_local() && comm_->size() > 1) {
          const unsigned long long big = 1ull << 62;
          unsigned long long v = big - (unsigned long long)std::max<int64_t>(0, cap);
          void* d = be_->alloc(8);
          be_->copy(d, &v, 8, CopyKind::H2D, kReduce);
          comm_token_wait(kReduce);
          comm_->allreduce(d, 1, RedType::U64, RedOp::Max, *be_, kReduce);
          comm_token_signal(kReduce);
          be_->copy(&v, d, 8, CopyKind::D2H, kReduce);
          be_->sync(kReduce);
          be_->release(d);
          cap = (int64_t)(big - v);
        }
        iter_cap = std::max(issued_, std::min<int64_t>(cfg_.iter_max, cap));
      }
      if (cfg_.progress_s > 0 && is_root() && now_s() - last_beat >= cfg_.progress_s) {
        // heartbeat: long convergence runs (1024^3 at eps 1e-5: ~2e5
        // iterations) stay visibly alive to launchers that kill silent jobs
        last_beat = now_s();
        const double el = last_beat - t0;
        std::fprintf(stderr, "heat3d: progress iteration %lld residual %.6e relative %.6e (eps %.3e) %.1f s, %.1f GLUPS\n",
                     (long long)hs.iter, hs.last_residual, hs.norm > 0 ? hs.last_residual / hs.norm : 0.0, hs.eps, el,
                     el > 0 ? (double)interior_points() * (double)(hs.iter - iter0) / el / 1e9 : 0.0);
        std::fflush(stderr);
      }
    }
    have_prev = true;
    pslot ^= 1;
    if (next_ckpt > 0 && issued_ >= next_ckpt && !stop) {
      HostState hs = state();
      if (!hs.done) save_checkpoint(cfg_.checkpoint_dir.empty() ? "checkpoint" : cfg_.checkpoint_dir);
      next_ckpt = issued_ + cfg_.checkpoint_every;
    }
    if (cfg_.verify_halo > 0 && issued_ >= next_verify) {
      const int bad = verify_halos();
      if (bad) {
        comm_->abort();
        HEAT3D_THROW("halo verification failed on " << bad << " face(s) after iteration " << issued_);
      }
      next_verify = issued_ + cfg_.verify_halo;
    }
  }
  be_->sync_all();
  comm_->check_async_error();
  const double t1 = now_s();
  HostState hs = state();
  if (cfg_.verbose > 0 && is_root()) {
    be_->copy(hstate_, dstate_, sizeof(DeviceState), CopyKind::D2H, kCompute);
    be_->sync(kCompute);
    for (int64_t it = printed; it < hs.iter; ++it)
      if (it % cfg_.verbose == 0 && it >= hs.iter - hstate_->hist_cap)
        std::printf("iteration %lld residual %.6e\n", (long long)it, hstate_->hist[it % hstate_->hist_cap]);
  }
  HEAT3D_CHECK(hs.fault != 2, "a device-side wait of a per-stream hipGraph timed out after "
                                   << cfg_.watchdog_s << " s (broken dependency or a stalled peer)");
  R.seconds = t1 - t0;
  R.fault = hs.fault != 0;
  R.converged = hs.done && !hs.fault;
  R.conv_iter = hs.conv_iter;
  R.issued = issued_;
  R.iterations = hs.done ? hs.conv_iter + 1 : issued_;
  R.norm = hs.norm;
  R.last_residual = hs.last_residual;
  // the final field is T^{iterations}: point the "current" parity at it
  if (hs.done) finalize_converged(hs.conv_iter);
  R.glups = R.seconds > 0 ? (double)interior_points() * (double)R.issued / R.seconds / 1e9 : 0.0;
  return R;
}

void Solver::compute_error(double* global_mean, double* local_mean) {
  be_->sync_all();
  const int p = cur();
  const std::size_t off = offsetof(DeviceState, error_sum);
  char* base = reinterpret_cast<char*>(dstate_);
  be_->memset(base + off, 0, 2 * sizeof(double), kCompute);
  for (std::size_t i = 0; i < local_.size(); ++i) {
    auto& l = local_[i];
    be_->error_accumulate(dt_, l.field[p], l.L, l.owned, l.sd.gstart, phys_.h[1], dstate_, kCompute);
    if (i == 0) {
      double e[2];
      be_->copy(e, base + off, sizeof(e), CopyKind::D2H, kCompute);
      be_->sync(kCompute);
      if (local_mean) *local_mean = e[1] > 0 ? e[0] / e[1] : 0.0;
    }
  }
  be_->sync(kCompute);
  if (!comm_->all_local() && comm_->size() > 1) {
    comm_->allreduce(base + off, 2, RedType::F64, RedOp::Sum, *be_, kCompute);
  }
  double e[2];
  be_->copy(e, base + off, sizeof(e), CopyKind::D2H, kCompute);
  be_->sync(kCompute);
  if (global_mean) *global_mean = e[1] > 0 ? e[0] / e[1] : 0.0;
}

int Solver::verify_halos() {
  be_->sync_all();
  if (issued_ == 0 || !has_halo_) return 0;
  // input buffer of the last iteration (or pair): its ghosts were filled by
  // that exchange from the neighbours' (unchanged) faces
  const int p = prv(cur());
  int nf = 0;
  for (auto& l : local_) nf += (int)l.faces.size();
  auto* dsum = static_cast<unsigned long long*>(be_->alloc(sizeof(unsigned long long) * 3 * nf));
  int q = 0;
  for (auto& l : local_)
    for (auto& io : l.faces) {
      // the regular depth: every exchange carries at least these planes
      be_->box_bitsum(dt_, l.field[p], l.L, io.g[0].send_box, dsum + 2 * q, kCompute);
      be_->box_bitsum(dt_, l.field[p], l.L, io.g[0].recv_box, dsum + 2 * q + 1, kCompute);
      ++q;
    }
  be_->sync(kCompute);
  std::vector<unsigned long long> h(3 * nf, 0);
  int bad = 0;
  if (comm_->all_local()) {
    be_->copy(h.data(), dsum, sizeof(unsigned long long) * 2 * nf, CopyKind::D2H, kCompute);
    be_->sync(kCompute);
    std::vector<int> base(local_.size(), 0);
    for (std::size_t i = 1; i < local_.size(); ++i) base[i] = base[i - 1] + (int)local_[i - 1].faces.size();
    for (std::size_t i = 0; i < local_.size(); ++i)
      for (std::size_t f = 0; f < local_[i].faces.size(); ++f) {
        const auto& io = local_[i].faces[f];
        const auto& nb = local_[io.peer_local];
        for (std::size_t g = 0; g < nb.faces.size(); ++g)
          if (nb.faces[g].face == opposite(io.face) && h[2 * (base[io.peer_local] + g)] != h[2 * (base[i] + f) + 1]) {
            std::fprintf(stderr, "heat3d: halo mismatch rank %d face %s\n", local_[i].sd.rank, face_name(io.face));
            ++bad;
          }
      }
  } else {
    // send my send-box checksum to each neighbour, receive theirs
    std::vector<Transfer> xs;
    q = 0;
    for (auto& l : local_)
      for (auto& io : l.faces) {
        Transfer s, r;
        s.src_rank = l.sd.rank;
        s.dst_rank = io.peer;
        s.src = dsum + 2 * q;
        s.bytes = 8;
        r.src_rank = io.peer;
        r.dst_rank = l.sd.rank;
        r.dst = dsum + 2 * nf + q;
        r.bytes = 8;
        xs.push_back(s);
        xs.push_back(r);
        ++q;
      }
    comm_->exchange(xs, *be_, kCompute);
    be_->sync(kCompute);
    be_->copy(h.data(), dsum, sizeof(unsigned long long) * 3 * nf, CopyKind::D2H, kCompute);
    be_->sync(kCompute);
    q = 0;
    for (auto& l : local_)
      for (auto& io : l.faces) {
        if (h[2 * nf + q] != h[2 * q + 1]) {
          std::fprintf(stderr, "heat3d: halo mismatch rank %d face %s (peer %d)\n", l.sd.rank,
                       face_name(io.face), io.peer);
          ++bad;
        }
        ++q;
      }
  }
  be_->release(dsum);
  return bad;
}

std::vector<std::pair<std::string, double>> Solver::phase_times() {
  std::vector<std::pair<std::string, double>> out = phase_acc_;
  for (auto& e : out) e.second /= std::max<int64_t>(1, phase_count_);
  return out;
}

void Solver::inject(int idx, int64_t i, int64_t j, int64_t k, double value, bool previous) {
  be_->sync_all();
  auto& l = local_.at(idx);
  HEAT3D_CHECK(i >= -1 && i <= l.sd.n[0] && j >= -1 && j <= l.sd.n[1] && k >= -1 && k <= l.sd.n[2],
               "inject index outside the ghosted block");
  be_->poke(dt_, l.field[previous ? prv(cur()) : cur()], l.L, i, j, k, value, kCompute);
  be_->sync(kCompute);
}

}  // namespace heat3d
