// heat3d-mi355x — the time-stepping engine.
//
// Reference call stack being replaced (heat3D.cu:541-1073):
// per iteration a full-volume host copy T0 = T, host face packing, 6 MPI
// Isends, a per-iteration GPU alloc/copy/launch/copy/free, blocking receives,
// host face/edge/corner updates, a host residual scan and a blocking
// MPI_Iallreduce of a break flag.
//
// Here one iteration t (parity p = t & 1, in = field[p], out = field[p^1]) is
//   compute stream : interior stencil (+ fused residual)            [A]
//   comm stream    : pack y/z faces -> exchange -> unpack -> shell stencils [B]
//   reduce stream  : allreduce(max residual) -> convergence check    [C]
// with A(t) || B(t), C(t) || A(t+1), B(t+1).  Kernels of iteration t+2 wait
// for C(t) and read its device flag: once converged they are no-ops, which
// leaves T^{t_conv+1} intact in field[(t_conv+1)&1].  The host polls a pinned
// copy of the flag every `check_every` iterations and never blocks the GPU
// pipeline per iteration (the reference synchronised every step,
// heat3D.cu:1062-1063).  Chunks of an even number of iterations are captured
// once into a hipGraph and replayed.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../comm/comm.hpp"
#include "../core/config.hpp"
#include "../core/decomp.hpp"
#include "backend.hpp"

namespace heat3d {

// Temporal blocking depth used when neither --temporal K nor --kernel2 tbK
// names one: fp64 3 (the lean kernel is HBM-bound at K = 3; K = 4 does not
// fit 16 waves x 128 VGPRs with 48-row tiles), fp32 3 (the packed-pair kernel,
// two columns per lane, has fp64's register shape: 48 x 128 tiles; 1450 GLUPS
// against 1288 for the one-column K = 4 kernel with 64-row tiles;
// profiles/kernel_sweep.md).
constexpr int kDefaultTemporal = 3;
constexpr int kDefaultTemporalF32 = 3;

struct RunResult {
  bool converged = false;
  bool fault = false;
  int64_t conv_iter = -1;    // 0-based iteration at which the criterion was met
  int64_t iterations = 0;    // iterations whose result is in the final field
  int64_t issued = 0;        // iterations enqueued (>= iterations when converged)
  double seconds = 0.0;      // wall time of the time loop (MPI_Wtime analogue)
  double norm = 1.0;
  double last_residual = 0.0;
  double error_mean = 0.0;   // global mean |T - y| over interior points
  double error_local = 0.0;  // this process's first subdomain (reference prints rank-0 local)
  double glups = 0.0;        // updated interior points x iterations / s (whole job)
};

struct HostState {
  double norm, eps, last_residual, error_sum, error_count;
  int64_t iter, conv_iter;
  int done, fault;
};

class Solver {
 public:
  // `process_rank` is the rank hosted by this process (ignored for LocalComm,
  // which hosts every rank).
  Solver(const Config& cfg, std::unique_ptr<Backend> be, std::unique_ptr<Comm> comm,
         std::array<int, 3> dims);
  ~Solver();
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  const Config& config() const { return cfg_; }
  const Decomposition& decomposition() const { return dec_; }
  const Physics& physics() const { return phys_; }
  Backend& backend() { return *be_; }
  Comm& comm() { return *comm_; }
  int process_rank() const { return local_.empty() ? 0 : local_[0].sd.rank; }
  bool is_root() const;
  int64_t interior_points() const { return (dec_.N[0] - 2) * (dec_.N[1] - 2) * (dec_.N[2] - 2); }
  std::string kernel_name() const {
    const std::string one = kspec_.resolved(cfg_.dtype).str();
    return tb_ ? kspec2_.resolved(cfg_.dtype).str() + "+" + one : one;
  }

  // (Re)initialise fields: analytic IC/BC (heat3D.cu:408-453) or restart.
  void initialize();
  // x-schedule autotuning of the interior sweeps (Config::autotune)
  void tune_schedules();
  // Untimed GPU warm-up that leaves the solver state untouched: `sweeps`
  // repetitions of the next sweep's interior, written into the buffer that
  // sweep will overwrite, without residual state (a sweep is idempotent).
  // Asynchronous on the compute stream; returns the sweeps issued.
  int preheat(int sweeps);
  // Full solve: iterate until converged or iter_max (heat3D.cu:541-1073).
  RunResult run();
  // Enqueue exactly n iterations without host polling (benchmarks); async.
  void step(int64_t n);
  // Capture (untimed) the hipGraph that step(n) will replay from the current
  // state, so that a timed step(n) only launches it.  No-op when graphs are off.
  void prepare_steps(int64_t n);
  void synchronize();
  HostState state();
  int64_t iterations_issued() const { return issued_; }
  // hipGraph launches so far (what actually ran, not the --graph request)
  int64_t graph_launches() const { return graph_launches_; }
  // The overlapped multi-stream schedule's per-stream hipGraphs: "n/a" (a
  // single-stream schedule), "off" (requested off, graphs off, or more than 4
  // ranks per GPU under auto), "on" (canary passed; details in
  // stream_graphs_note()), "unverified" (--graph-canary 0) or "fallback" (the
  // canary timed out or ran > 2x eager on some rank: eager for the job).
  const std::string& stream_graphs_state() const { return sg_state_; }
  const std::string& stream_graphs_note() const { return sg_note_; }
  // processes sharing this rank's GPU, as the launcher's environment tells
  int ranks_per_device() const { return ranks_per_device_; }
  // full sweeps check convergence from their last residual (residual_last_ok)
  bool monotone_check() const { return rl_; }

  // Error vs analytic steady state (heat3D.cu:1093-1106, with a true global
  // mean instead of rank-0's local value).  Uses the current field.
  void compute_error(double* global_mean, double* local_mean);

  // Field access.  gather_global fills `out` (N0*N1*N2 values as double,
  // z fastest) on the root process only; returns false elsewhere.
  bool gather_global(std::vector<double>* out);
  // Local subdomain (index into local_ranks()) owned+ghost values as double.
  std::vector<double> local_field(int local_idx, bool with_ghosts);
  int num_local() const { return (int)local_.size(); }
  const Subdomain& local_subdomain(int i) const { return local_[i].sd; }
  const Layout& local_layout(int i) const { return local_[i].L; }
  // current field buffer of a local subdomain (device pointer on HIP)
  void* local_field_ptr(int i) { return local_[i].field[cur()]; }
  // True when iterations run as K-step temporally blocked sweeps (single
  // subdomain, or x slabs with K-plane halos); K = temporal_steps().
  bool temporal_blocking() const { return tb_; }
  int temporal_steps() const { return K_; }
  // field buffers per subdomain (3 = lagged convergence check of overlapped sweeps)
  int field_buffers() const { return nbuf_; }
  // ghost depth per axis (K on split axes with temporal blocking, K+1 when
  // long sweeps cross the halos) and whether they do
  std::array<int64_t, 3> ghost_depth() const { return {hd_[0], hd_[1], hd_[2]}; }
  bool long_halo_sweeps() const { return long_halo_; }
  // the overlapped sweeps' interior and boundary pieces of local subdomain i
  // (lo0, hi0, lo1, hi1, lo2, hi2 each)
  std::vector<std::array<int64_t, 6>> sweep_pieces(int i) const {
    std::vector<std::array<int64_t, 6>> out;
    auto add = [&](const Box& b) { out.push_back({b.lo[0], b.hi[0], b.lo[1], b.hi[1], b.lo[2], b.hi[2]}); };
    add(local_.at(i).tb_interior);
    for (const Box& b : local_.at(i).tb_boundary) add(b);
    return out;
  }
  // remainder policy: which n mod K run as long sweeps, and the start-up
  // sweep timings that decided it (empty when not measured)
  unsigned long_remainders() const { return long_rem_; }
  bool long_major() const { return long_major_; }
  const std::vector<std::pair<std::string, double>>& sweep_costs() const { return sweep_costs_; }
  // HBM preflight (constructor): bytes this solver allocates for its local
  // ranks (fields + face staging), and the backend's free / total memory
  // just before those allocations (0 when the backend cannot tell)
  std::size_t planned_bytes() const { return planned_bytes_; }
  std::size_t mem_free_before() const { return mem_free_before_; }
  std::size_t mem_total() const { return mem_total_; }

  // Output / checkpoint.
  void write_tecplot(const std::string& path, const std::string& layout);
  // per-rank zones ("owned" layout), written in parallel at computed offsets
  void write_tecplot_zones(const std::string& path);
  void save_checkpoint(const std::string& dir);
  void load_checkpoint(const std::string& dir);

  // Per-phase timing (ms, averaged over timed iterations) when enabled.
  // Diagnostic: every iteration is synchronised, graphs are off.
  void set_phase_timing(bool on) {
    phase_timing_ = on;
    phase_acc_.clear();
    phase_count_ = 0;
  }
  std::vector<std::pair<std::string, double>> phase_times();

  // Schedule profile of the production sweep pipeline (diagnostic, run it
  // outside any timed window): issues n more temporally blocked sweeps eagerly
  // with timing events at the phase boundaries of every stream and returns
  // per-sweep means in ms (interior, halo, boundary, all-reduce, check, sweep
  // period, compute-stream idle, boundary tail after the interior) plus the
  // fraction of the halo + boundary chain that ran while the interior did.
  // Unlike set_phase_timing() nothing is synchronised between sweeps, so the
  // numbers describe the overlapped schedule as it runs.
  std::vector<std::pair<std::string, double>> profile_sweeps(int n);

  // Link probe (the decomposition choice of a multi-GPU job): every rank
  // exchanges `bytes` with each ring neighbour (ranks r - 1 and r + 1, the
  // two x faces of a slab) at once, `reps` times after a warm-up, through the
  // run's transport; returns the slowest rank's best one-way rate per link in
  // GB/s (an all-reduce: the same value on every rank), 0 for one rank.
  double link_probe(std::size_t bytes, int reps);

  // Race detection: compare order-independent checksums of every face sent
  // in the last exchange with the ghost layer the neighbour received.
  // Returns the number of mismatching faces (0 = consistent).
  int verify_halos();

  // Fault injection for tests: write `value` into a local owned point.
  // `previous` targets the other ping-pong buffer (the last iteration's input).
  void inject(int local_idx, int64_t i, int64_t j, int64_t k, double value, bool previous = false);

 private:
  // One face's exchange at one halo depth: the K-plane halo of regular
  // sweeps (dv = 0), the (K+1)-plane halo of long sweeps (dv = 1; the same as
  // dv = 0 without long_halo_).  Boxes in local coordinates.
  struct FaceGeom {
    Box send_box, recv_box;
    int64_t send_off = 0, recv_off = 0, elems = 0;  // contiguous x faces: in place
  };
  struct FaceIO {
    Face face;
    int peer;
    FaceGeom g[2];
    bool contiguous = false;    // x faces: whole planes sent in place
    void* sendbuf = nullptr;    // staging for packed faces (sized for the deepest halo)
    void* recvbuf = nullptr;
    int peer_local = -1;        // LocalComm: index of the neighbour in local_
  };
  struct Local {
    Subdomain sd;
    Layout L;
    void* field[3] = {nullptr, nullptr, nullptr};  // nbuf_ of them in use
    Box owned, interior;
    std::vector<Box> shell;
    std::vector<FaceIO> faces;
    // temporally blocked sweeps with deep x halos: interior planes [K, n0-K)
    // (need no halo), K-plane boundary slabs, u range widened into the halos
    Box tb_interior;
    std::vector<Box> tb_boundary;
    // the same for long sweeps of depth K+1 across halos (long_halo_)
    Box tb_interior_long;
    std::vector<Box> tb_boundary_long;
    int64_t ux[2] = {0, -1};
    int64_t uy[2] = {0, -1}, uz[2] = {0, -1};  // y / z update ranges (deep y / z halos)
  };

  void setup_faces();
  // initialize(): the analytic IC (or nothing, before a restart) into every
  // field buffer, and the device state / schedule counters / events of
  // iteration 0 (restart: of the checkpoint)
  void init_fields();
  void reset_state();
  // Start-up canary of the per-stream graphs (initialize(), every rank at the
  // same point): one schedule cycle eagerly, then the same cycle as per-stream
  // graphs with the device-side waits' timeout cut to --graph-canary; a
  // timed-out wait or a replay > 2x the eager time on any rank (one vote)
  // turns the graphs off for the job.  The fields are re-initialised after.
  void canary_stream_graphs();
  void set_wait_timeout(double seconds);
  bool stream_graphs_enabled() const;
  // fault 2 (a timed-out device-side wait) after per-stream graph launches
  void check_graph_fault();
  // one single-step iteration: residual slot / event parity p, input buffer bi
  void enqueue_iteration(int p, int bi);
  // K iterations in one temporally blocked sweep from buffer bi
  // thick: boundary layers K+1 deep (the long sweeps' pieces) for a K-step
  // sweep that a long sweep follows (its K+1-deep halo sends the planes
  // this sweep writes, which must come from the boundary slabs, not the
  // interior the halo does not wait for)
  void enqueue_multi(int bi, int Kp = 0, bool thick = false);
  // dv: halo depth variant (FaceGeom), 1 = the K+1 planes of a long sweep
  void enqueue_halo(int bi, StreamId s, int dv = 0);
  template <typename Pred>
  void enqueue_halo_phase(int bi, StreamId s, int dv, Pred in_phase);
  void join_pipeline();      // every stream waits for every pipeline event
  // Collective ordering chain (ordered_collectives comms, > 1 rank): every
  // exchange / all-reduce waits for the previous one's completion event, so
  // each GPU runs the job's collectives in one total order, the host issue
  // order, which is identical on all ranks.
  void comm_token_wait(StreamId s);
  void comm_token_signal(StreamId s);
  // all-reduce + check of one sweep (residual slots slot0 .. slot0+Kp-1)
  void reduce_and_check(StreamId s, int slot0, int Kp, int prof = -1, bool last_only = false);
  // the non-overlapped sweep of a single-subdomain run checks convergence in
  // its last workgroup (StencilParams::fuse_check; --no-fused-check: off)
  bool fused_check() const;
  // ... from the last residual of each full sweep (kResidualLastOnly): fused
  // check, no residual history, and an update whose max-norm residual cannot
  // grow (1 - 2(Dx + Dy + Dz) >= 0: T' is a convex combination of T's 7
  // points, so max|T'' - T'| <= max|T' - T| with fixed boundary values)
  bool residual_last_ok() const;
  KernelSpec last_only(const KernelSpec& ks) const;
  // a sweep with the last residual only set done: replay it with all K
  // residuals (same fields, rewritten bit for bit) into a scratch state and
  // put the first converged (or faulted) iteration into the device state
  void resolve_coarse();
  // sweeps of depth Kp >= 2 after iteration 0 run ks_last_[Kp] where rl_d_[Kp]
  // (residual_last_ok and the variant exists); rl_ = rl_d_[K_]
  bool rl_ = false;
  bool rl_d_[8] = {};
  bool long_major_ = false;          // K+1 sweeps cheaper per step (calibrate_remainders, long_sweeps_for)
  KernelSpec ks_last_[8];
  KernelSpec rl_pick_[8];            // per depth: the variant the start-up timing kept
  // lagged overlapped sweeps: the all-reduce of sweep q is issued after the
  // halo of sweep q+1 (see enqueue_multi); flush issues a pending one
  void flush_pending_reduce();
  unsigned long long allreduce_sum_u64(unsigned long long v);
  bool graphs_allowed() const;
  int graph_len_for(int64_t n) const;
  // Sweeps of depth K+1 that absorb the remainder of a chunk of n steps that
  // is not a multiple of K (single subdomain, lean kernel): n = a K + b (K+1)
  // costs a + b HBM passes where a K-sweep + a partial one would cost one more.
  int long_sweeps_for(int64_t n) const;
  bool multi_stream() const { return tb_ ? tb_overlap_ : overlap_; }
  // buffer holding T^{issued_}; a step or a K-step sweep reads cur() and
  // writes nxt(cur())
  int cur() const { return cur_; }
  int nxt(int b) const { return b + 1 == nbuf_ ? 0 : b + 1; }
  int prv(int b) const { return b == 0 ? nbuf_ - 1 : b - 1; }
  void record_segment(int64_t start, int len, int inbuf);
  void finalize_converged(int64_t conv_iter);
  void ev_record(int id, StreamId s);
  void ev_wait(StreamId s, int id);
  void run_chunk(int64_t n);
  // graph replaying G iterations from the current (buffer, parity) state
  struct GraphEntry {
    void* exec = nullptr;
    int G = 0, kind = 1, buf = 0, parity = 0, sparity = 0;
    bool first = false;  // captured at iteration 0 (its first sweep computes every residual)
  };
  GraphEntry* find_graph(int G, int kind = 0);
  GraphEntry* build_graph(int G, int kind = 0);
  int long_graph_cap() const;
  void destroy_graphs();
  InitParams init_params(const Local& l) const;

  Config cfg_;
  std::unique_ptr<Backend> be_;
  std::unique_ptr<Comm> comm_;
  Decomposition dec_;
  Physics phys_;
  KernelSpec kspec_;
  std::vector<Local> local_;
  bool has_halo_ = false;  // any face with a neighbour on any local subdomain
  bool overlap_ = true;
  bool tb_overlap_ = false;   // sweeps: interior || (deep halo -> boundary slabs)
  bool long_slab_ = false;    // x-slab share whose interior hides the halo chain (no CU reservation)
  int64_t hd_[3] = {1, 1, 1}; // ghost depth per axis (K on split axes with temporal blocking, K+1 with long_halo_)
  int64_t xd_[3] = {1, 1, 1}; // regular exchange depth per axis (K on split axes with temporal blocking)
  // Long sweeps (depth K+1) across halos: ghosts allocated K+1 deep on split
  // axes, exchanged K+1 deep before a long sweep only; step counts that are
  // not multiples of K end in long sweeps instead of a partial K-1 sweep
  bool long_halo_ = false;
  int slot_stride_ = 1;       // residual slots per sweep bank of the lagged schedule
  // remainder policy (long_sweeps_for): bit r set = a step count with n mod K
  // = r ends in r long sweeps, else in a partial sweep of r steps
  unsigned long_rem_ = ~0u;
  // kernel of a sweep of depth Kp != K (partial / long): the family default,
  // or the variant the start-up timing kept (depth_spec_[Kp] where depth_set_)
  KernelSpec depth_spec_[8];
  bool depth_set_[8] = {};
  KernelSpec spec_for_depth(int Kp) const;
  std::vector<std::pair<std::string, double>> sweep_costs_;  // start-up timings (ms per sweep)
  void calibrate_remainders();
  bool pick_sweep_form() const;
  KernelSpec pair_form() const;
  int last_bnd_ = 0;          // boundary-layer depth of the last overlapped sweep (0: none pending)
  bool ordered_halo_ = false; // axis-ordered exchange filling edges / corners (deep y / z halos)
  int last_kind_ = 0;         // 1 = single step, 2 = pair: last enqueued schedule
  DType dt_;
  std::size_t esize_;

  DeviceState* dstate_ = nullptr;   // device
  DeviceState* rstate_ = nullptr;   // device scratch of resolve_coarse (allocated on first use)
  DeviceState* hstate_ = nullptr;   // pinned host mirror
  int64_t issued_ = 0;              // iterations enqueued so far (absolute index)
  int cur_ = 0;               // buffer holding T^{issued_}
  // Field buffers: 2 (ping-pong), or 3 for overlapped x-slab sweeps, where the
  // convergence check of sweep q (all-reduce + check kernel) is lagged: sweep
  // q+1 runs speculatively into the third buffer and only sweep q+2, which
  // overwrites sweep q's input (needed for a rollback), waits for it.
  int nbuf_ = 2;
  std::size_t planned_bytes_ = 0, mem_free_before_ = 0, mem_total_ = 0;
  void preflight_memory();
  bool lag_ = false;
  int64_t nsweep_ = 0;            // overlapped sweeps issued (event / residual-slot parity)
  double fake_allreduce_us_ = 0;  // diagnostic: emulated all-reduce latency (virtual ranks)
  bool tb_ = false;           // K-step temporal blocking active
  int K_ = 1;                 // iterations per sweep
  KernelSpec kspec2_;
  struct Segment {
    int64_t start;
    int len;    // 1 = single step, K = temporally blocked sweep
    int inbuf;  // buffer read by the segment
  };
  std::vector<Segment> segs_;       // ring of recent segments (for convergence rollback)
  std::size_t seg_head_ = 0;

  // events: 0..1 int[p], 2..3 bnd[p], 4..5 check[p], 6 fork, 7 join comm, 8 join red, 9..10 poll
  enum { EV_INT = 0, EV_BND = 2, EV_CHK = 4, EV_FORK = 6, EV_JCOMM = 7, EV_JRED = 8, EV_POLL = 9,
         EV_T0 = 11, EV_T1 = 12, EV_TOKEN = 13, EV_COUNT = 16 };
  bool chain_ = false;              // collective ordering chain active
  struct PendingReduce {
    bool valid = false;
    int q = 0, slot0 = 0, Kp = 0;
    int prof = -1;  // profiled sweep index (profile_sweeps)
    bool last_only = false;  // the interior computed only the last residual
  } pending_;
  Event ev_[EV_COUNT] = {};
  Event cur_ev_[EV_COUNT] = {};     // event currently standing for each id
  std::vector<Event> cap_pool_;     // fresh events for records inside a capture
  std::size_t cap_next_ = 0;
  bool ev_valid_[EV_COUNT] = {};
  bool capturing_ = false;

  std::vector<GraphEntry> graphs_;  // small cache, keyed by (G, kind, buf, parities)
  bool graph_failed_ = false;
  int64_t graph_launches_ = 0;
  bool force_eager_ = false;        // canary: the eager reference chunk
  bool sg_fallback_ = false;        // the canary turned the per-stream graphs off (sticky)
  bool sg_unchecked_ = false;       // per-stream graphs launched since the last fault check
  int ranks_per_device_ = 1;
  std::string sg_state_ = "n/a", sg_note_;

  bool phase_timing_ = false;
  std::vector<std::pair<std::string, double>> phase_acc_;
  int64_t phase_count_ = 0;
  Event tev_[8] = {};
  void accumulate_phase_times();

  // profile_sweeps: events per profiled sweep, recorded only while prof_on_
  enum { PE_INT0, PE_INT1, PE_HALO0, PE_XCHG0, PE_HALO1, PE_BND0, PE_BND1, PE_RED0, PE_REDX, PE_CHK1, PE_COUNT };
  bool prof_on_ = false;
  int prof_idx_ = -1;                 // sweep being issued
  std::vector<Event> prof_ev_;        // PE_COUNT per sweep
  std::vector<unsigned> prof_set_;    // bit mask of the events recorded per sweep
  void prof_record(int sweep, int id, StreamId s);
};

// Where one rank of a job runs: its rank, the job size, the GPU it binds, and
// how it meets its peers (rank 0's bootstrap address / port).  With a
// non-empty rccl_uid the RCCL communicator is created directly from it (the
// ranks of one process share it: ncclCommInitAll semantics, one host thread
// per GPU) instead of through the TCP bootstrap.
struct RankPlacement {
  int rank = 0, size = 1, local_rank = 0;
  int device = -1;  // -1: local_rank modulo the visible devices
  std::string master = "127.0.0.1";
  int bootstrap_port = 29501;
  std::string rccl_uid;
};

// Communicator options from the run configuration
inline RcclOptions rccl_options(const Config& c) {
  RcclOptions o;
  o.shared = c.rccl_shared;
  o.graph = c.rccl_graph;
  // RCCL's P2P channel pool: its default unless asked for.  (Round 5 capped
  // it at the reserved CUs for every RCCL job, before the communicator knew
  // the reservation the solver would choose, and never timed the cap on real
  // xGMI links: opt-in until a multi-GPU A/B shows it does not cost halo rate.)
  o.p2p_channels = c.rccl_p2p_channels > 0 ? c.rccl_p2p_channels : 0;
  return o;
}
inline PhantomOptions phantom_options(const Config& c) {
  PhantomOptions o;
  o.gbps = c.phantom_gbps;
  o.allreduce_us = c.phantom_allreduce_us;
  o.channels = c.phantom_channels;
  o.overlap_copies = c.phantom_overlap;
  o.paced = c.phantom_paced;
  o.rccl_footprint = c.phantom_rccl_footprint;
  o.allreduce_channels = c.phantom_allreduce_channels;
  return o;
}

// Build a Solver for one rank: chooses backend, comm (RCCL / socket through
// the bootstrap, LocalComm for --virtual-ranks), decomposition.
std::unique_ptr<Solver> make_solver(const Config& cfg, const RankPlacement& where);

// Same, placement from the environment: RANK/WORLD_SIZE/LOCAL_RANK/
// MASTER_ADDR/MASTER_PORT (torchrun / mpirun style).
std::unique_ptr<Solver> make_solver_from_env(const Config& cfg);
// This process's rank as the launcher tells it: RANK (torchrun),
// OMPI_COMM_WORLD_RANK (Open MPI) or PMI_RANK (MPICH hydra); 0 without one.
int rank_from_env();

}  // namespace heat3d
