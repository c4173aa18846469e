// heat3d-mi355x — Python bindings (pybind11, no torch headers).
//
// Exposes the native runtime (Solver, topology, decomposition, RCCL/socket
// bootstrap helpers) and the individual gfx950 / CPU kernels on raw pointers
// so that the Python package can drive them on torch tensors
// (tensor.data_ptr(), torch.cuda.current_stream().cuda_stream).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include <hip/hip_runtime.h>

#include "../comm/comm.hpp"
#include "../comm/net.hpp"
#include "../core/config.hpp"
#include "../core/decomp.hpp"
#include "../compat/reference_scheme.hpp"
#include "../runtime/solver.hpp"

namespace py = pybind11;
using namespace heat3d;

namespace {

Config parse_args(const std::vector<std::string>& args) {
  std::vector<const char*> av;
  av.push_back("heat3d");
  for (auto& a : args) av.push_back(a.c_str());
  return Config::parse((int)av.size(), av.data());
}

Box to_box(const std::array<int64_t, 6>& b) {
  Box r;
  for (int a = 0; a < 3; ++a) {
    r.lo[a] = b[2 * a];
    r.hi[a] = b[2 * a + 1];
  }
  return r;
}

Layout to_layout(const std::array<int64_t, 3>& n, int64_t esize, int64_t gx = 1, int64_t gy = 1, int64_t gz = 1) {
  int64_t nn[3] = {n[0], n[1], n[2]};
  return Layout::make(nn, esize, gx, gy, gz);
}

py::dict layout_dict(const Layout& L) {
  py::dict d;
  d["n"] = py::make_tuple(L.n[0], L.n[1], L.n[2]);
  d["sx"] = L.sx;
  d["sy"] = L.sy;
  d["zoff"] = L.zoff;
  d["origin"] = L.origin;
  d["elems"] = L.elems;
  d["esize"] = L.esize;
  d["gx"] = L.gx;
  return d;
}

py::dict sub_dict(const Subdomain& s) {
  py::dict d;
  d["rank"] = s.rank;
  d["coords"] = py::make_tuple(s.coords[0], s.coords[1], s.coords[2]);
  d["n"] = py::make_tuple(s.n[0], s.n[1], s.n[2]);
  d["gstart"] = py::make_tuple(s.gstart[0], s.gstart[1], s.gstart[2]);
  py::list nb;
  for (int f = 0; f < kNumFaces; ++f) nb.append(s.neighbors[f]);
  d["neighbors"] = nb;
  Box e = s.extended_global();
  d["extended"] = py::make_tuple(e.lo[0], e.hi[0], e.lo[1], e.hi[1], e.lo[2], e.hi[2]);
  return d;
}

py::array_t<double> to_numpy(std::vector<double>&& v, std::vector<py::ssize_t> shape) {
  auto* heap = new std::vector<double>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete static_cast<std::vector<double>*>(p); });
  std::vector<py::ssize_t> strides(shape.size());
  py::ssize_t st = sizeof(double);
  for (int i = (int)shape.size() - 1; i >= 0; --i) {
    strides[i] = st;
    st *= shape[i];
  }
  return py::array_t<double>(shape, strides, heap->data(), owner);
}

std::unique_ptr<Solver> create_solver(const std::vector<std::string>& args, int rank, int size,
                                      const std::string& comm_kind, py::bytes unique_id,
                                      int listen_fd, const std::vector<std::string>& addrs,
                                      int device) {
  Config cfg = parse_args(args);
  BackendKind bk = cfg.backend;
  if (bk == BackendKind::Auto) bk = hip_device_count() > 0 ? BackendKind::Hip : BackendKind::Cpu;
  int dev = device >= 0 ? device : (cfg.device >= 0 ? cfg.device : 0);
  std::unique_ptr<Backend> be = bk == BackendKind::Hip ? make_hip_backend(dev) : make_cpu_backend(cfg.cpu_threads);
  std::unique_ptr<Comm> comm;
  int nranks = 1;
  if (comm_kind == "local" || comm_kind == "none") {
    nranks = cfg.virtual_ranks;
    comm = make_local_comm(nranks);
  } else if (comm_kind == "rccl") {
    HEAT3D_CHECK(bk == BackendKind::Hip, "rccl comm needs the HIP backend");
    comm = make_rccl_comm(rank, size, std::string(unique_id), dev, rccl_options(cfg));
    nranks = size;
  } else if (comm_kind == "phantom") {
    comm = make_phantom_comm(rank, size, phantom_options(cfg));
    nranks = size;
  } else if (comm_kind == "socket" || comm_kind == "staged") {
    // a GPU backend always stages through host memory; "staged" forces the
    // wrapper on the CPU backend too (tests of the staging logic without a GPU)
    comm = make_socket_comm_from_table(rank, size, listen_fd, addrs);
    if (bk == BackendKind::Hip || comm_kind == "staged") comm = make_staged_comm(std::move(comm));
    nranks = size;
  } else {
    throw UsageError("unknown comm kind '" + comm_kind + "'");
  }
  std::array<int, 3> fixed = {0, 0, 0};
  if (cfg.decomp[0] > 0) fixed = cfg.decomp;
  auto dims = dims_create(nranks, fixed);
  return std::unique_ptr<Solver>(new Solver(cfg, std::move(be), std::move(comm), dims));
}

DType dt_of(const std::string& s) { return parse_dtype(s); }

StencilParams sparams(int64_t in_ptr, int64_t out_ptr, const std::array<int64_t, 3>& n,
                      int64_t esize, const std::array<int64_t, 6>& box,
                      const std::array<double, 3>& D, int64_t state_ptr, int slot) {
  StencilParams p;
  p.in = reinterpret_cast<const void*>(in_ptr);
  p.out = reinterpret_cast<void*>(out_ptr);
  p.L = to_layout(n, esize);
  p.box = to_box(box);
  for (int a = 0; a < 3; ++a) p.D[a] = D[a];
  p.state = reinterpret_cast<DeviceState*>(state_ptr);
  p.slot = slot;
  return p;
}

// HEAT3D_SEGV_TRACE=1: print the native backtrace on SIGSEGV/SIGBUS/SIGFPE
// (no debugger on the GPU boxes), then re-raise with the default action.
void segv_trace(int sig) {
  void* frames[64];
  int n = backtrace(frames, 64);
  const char msg[] = "\nheat3d: fatal signal, native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void install_segv_trace() {
  const char* e = std::getenv("HEAT3D_SEGV_TRACE");
  if (!e || !*e || e[0] == '0') return;
  for (int s : {SIGSEGV, SIGBUS, SIGFPE, SIGILL}) signal(s, segv_trace);
}

}  // namespace

PYBIND11_MODULE(_heat3d, m) {
  install_segv_trace();
  m.doc() = "heat3d-mi355x native runtime (HIP/gfx950 kernels, RCCL/socket comm, solver)";
  auto native_error = py::register_exception<Error>(m, "NativeError", PyExc_RuntimeError);
  py::register_exception<UsageError>(m, "UsageError", native_error.ptr());

  m.def("device_count", &hip_device_count);
  // the lean kernel's z tile stride for a box (host model; tests/test_temporal_cpu.py)
  m.def("lean_z_stride", [](int64_t nx, int64_t ny, int64_t nz, int K, int esize, int TY, int slots, int U) {
    return heat3d::hip::lean_z_stride(nx, ny, nz, K, esize, TY, slots, U, 0);
  });
  // the x plan of a sweep and its modelled makespan (plane steps per slot)
  m.def("x_plan", [](int64_t nx, int64_t tiles, int slots, int fill, int U, int seg) {
    const heat3d::hip::XPlanInfo p = heat3d::hip::describe_xplan(nx, tiles, slots, fill, U, seg);
    py::dict d;
    d["seg"] = p.seg;
    d["n1"] = p.n1;
    d["r"] = p.r;
    d["split"] = p.split;
    d["nb2"] = p.nb2;
    d["makespan"] = p.makespan;
    d["ideal"] = (double)tiles * (double)(nx + fill) / slots;
    return d;
  }, py::arg("nx"), py::arg("tiles"), py::arg("slots"), py::arg("fill"), py::arg("U"), py::arg("seg") = 0);
  // the start-up tuner's model-best fixed x segments (any length)
  m.def("best_fixed_segments", &heat3d::hip::best_fixed_segments, py::arg("nx"), py::arg("tiles"), py::arg("slots"),
        py::arg("fill"), py::arg("U"), py::arg("count") = 2);
  // x schedules chosen by timing at solver start-up (Config::autotune)
  m.def("tuned_schedules", []() {
    py::list out;
    for (const auto& t : heat3d::hip::tuned_schedules()) {
      py::dict d;
      d["kernel"] = t.kernel;
      d["nx"] = t.nx;
      d["ny"] = t.ny;
      d["nz"] = t.nz;
      d["zs"] = t.zs;
      d["L"] = t.L;
      d["ms"] = t.ms;
      d["ms_model"] = t.ms_model;
      d["candidates"] = t.candidates;
      out.append(d);
    }
    return out;
  });
  m.def("pair_z_stride", [](int64_t nx, int64_t ny, int64_t nz, int K, int TY, int slots, int U, int esize) {
    return heat3d::hip::pair_z_stride(nx, ny, nz, K, TY, slots, U, 0, esize);
  }, py::arg("nx"), py::arg("ny"), py::arg("nz"), py::arg("K"), py::arg("TY"), py::arg("slots"), py::arg("U"),
     py::arg("esize") = 4);
  // a kernel spec with its per-dtype defaults filled in, as the solver
  // launches it (tests/test_temporal_cpu.py)
  m.def("kernel_spec_resolved", [](const std::string& spec, const std::string& dtype) {
    return heat3d::KernelSpec::parse(spec).resolved(dtype == "fp32" ? heat3d::DType::F32 : heat3d::DType::F64).str();
  });
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def("rccl_version", &rccl_version);
  // the HIP runtime / RCCL this process is bound to (bench JSON "runtime")
  m.def("runtime_info", []() {
    const HipRuntimeInfo h = hip_runtime_info();
    py::dict d;
    d["hip_runtime_version"] = h.runtime_version;
    d["hip_driver_version"] = h.driver_version;
    d["hip_library"] = h.library;
    d["sync_wait"] = h.sync_wait;
    d["rccl_version"] = rccl_version();
    d["rccl_library"] = rccl_library_path();
    return d;
  });
  m.def("device_synchronize", [](int device) {
    py::gil_scoped_release nogil;
    hip_device_synchronize(device);
  });
  // Host collectives of a job without torch (bench.py's ranks): a star of TCP
  // connections to rank 0 (net::Bootstrap), kept open for the job.
  py::class_<net::Bootstrap>(m, "HostGroup")
      .def(py::init([](int rank, int size, const std::string& master, int port, double timeout_s) {
             py::gil_scoped_release nogil;
             return std::unique_ptr<net::Bootstrap>(new net::Bootstrap(rank, size, master, port, timeout_s));
           }),
           py::arg("rank"), py::arg("size"), py::arg("master"), py::arg("port"), py::arg("timeout_s") = 600.0)
      .def("allgather", [](net::Bootstrap& b, py::bytes blob) {
        std::string s(blob);
        std::vector<std::string> all;
        {
          py::gil_scoped_release nogil;
          all = b.allgather(s);
        }
        py::list out;
        for (auto& a : all) out.append(py::bytes(a));
        return out;
      })
      .def("barrier", [](net::Bootstrap& b) {
        py::gil_scoped_release nogil;
        b.barrier();
      })
      .def_property_readonly("rank", &net::Bootstrap::rank)
      .def_property_readonly("size", &net::Bootstrap::size);
  // Which CUs a stream created with a CU mask reaches: runs the placement
  // probe on hipExtStreamCreateWithCUMask(mask) (an empty mask: a plain
  // stream) and returns the distinct (XCC << 8 | SE/SH/CU) ids seen.
  m.def("cu_mask_probe", [](int device, std::vector<uint32_t> mask, int blocks) {
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
    hipStream_t st = nullptr;
    if (mask.empty()) {
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) throw std::runtime_error("stream");
    } else if (hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()) != hipSuccess) {
      throw std::runtime_error("hipExtStreamCreateWithCUMask failed");
    }
    unsigned* d = nullptr;
    if (hipMalloc(&d, sizeof(unsigned) * blocks) != hipSuccess) throw std::runtime_error("hipMalloc");
    heat3d::hip::cu_probe(d, blocks, 50.0, st);
    std::vector<unsigned> h(blocks);
    if (hipMemcpyAsync(h.data(), d, sizeof(unsigned) * blocks, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      throw std::runtime_error("probe failed");
    (void)hipFree(d);
    (void)hipStreamDestroy(st);
    std::sort(h.begin(), h.end());
    h.erase(std::unique(h.begin(), h.end()), h.end());
    return h;
  }, py::arg("device"), py::arg("mask"), py::arg("blocks") = 8192);
  // Executes RcclComm::exchange / allreduce on a one-rank communicator: every
  // transfer is a send and a receive to self inside one RCCL group (sizes that
  // are and are not multiples of 8 bytes), plus a padded K-deep x halo plane of
  // a ghosted Layout moved in place between two fields, as the solver sends
  // x faces.  Returns per-transfer byte equality and the all-reduce results.
  m.def("rccl_self_exchange", [](int device, std::vector<int64_t> sizes, std::array<int64_t, 3> n, int depth) {
    auto be = make_hip_backend(device);
    auto comm = make_rccl_comm(0, 1, rccl_unique_id(), device);
    std::vector<Transfer> xs;
    std::vector<std::vector<unsigned char>> want;
    std::vector<void*> dsts, bufs;
    auto pattern = [](std::size_t bytes, unsigned seed) {
      std::vector<unsigned char> h(bytes);
      for (std::size_t i = 0; i < bytes; ++i) h[i] = (unsigned char)((i * 131u + seed * 17u + (i >> 8)) & 0xff);
      return h;
    };
    for (std::size_t q = 0; q < sizes.size(); ++q) {
      const std::size_t b = (std::size_t)sizes[q];
      void* src = be->alloc(b);
      void* dst = be->alloc(b);
      auto h = pattern(b, (unsigned)q + 1);
      be->copy(src, h.data(), b, CopyKind::H2D, kComm);
      be->memset(dst, 0xEE, b, kComm);
      be->sync(kComm);
      Transfer t;
      t.src_rank = t.dst_rank = 0;
      t.src = src;
      t.dst = dst;
      t.bytes = b;
      xs.push_back(t);
      want.push_back(h);
      dsts.push_back(dst);
      bufs.push_back(src);
      bufs.push_back(dst);
    }
    // padded x halo: planes [n0-depth, n0) of field A into ghost planes
    // [-depth, 0) of field B, whole planes (ghost rows and row padding included)
    int64_t nn[3] = {n[0], n[1], n[2]};
    const Layout L = Layout::make(nn, 8, depth, 1, 1);
    void* fa = be->alloc(L.bytes());
    void* fb = be->alloc(L.bytes());
    auto ha = pattern(L.bytes(), 99);
    be->copy(fa, ha.data(), L.bytes(), CopyKind::H2D, kComm);
    be->memset(fb, 0xEE, L.bytes(), kComm);
    be->sync(kComm);
    const std::size_t pb = (std::size_t)(depth * L.sx * 8);
    Transfer t;
    t.src_rank = t.dst_rank = 0;
    t.src = static_cast<char*>(fa) + L.plane_offset(n[0] - depth) * 8;
    t.dst = static_cast<char*>(fb) + L.plane_offset(-depth) * 8;
    t.bytes = pb;
    xs.push_back(t);
    want.emplace_back(ha.begin() + L.plane_offset(n[0] - depth) * 8, ha.begin() + L.plane_offset(n[0] - depth) * 8 + pb);
    dsts.push_back(t.dst);
    comm->exchange(xs, *be, kComm);
    be->sync(kComm);
    comm->check_async_error();
    py::list ok;
    for (std::size_t q = 0; q < xs.size(); ++q) {
      std::vector<unsigned char> got(xs[q].bytes);
      be->copy(got.data(), dsts[q], xs[q].bytes, CopyKind::D2H, kComm);
      be->sync(kComm);
      ok.append(got == want[q]);
    }
    // the planes around the halo must be untouched
    std::vector<unsigned char> whole(L.bytes());
    be->copy(whole.data(), fb, L.bytes(), CopyKind::D2H, kComm);
    be->sync(kComm);
    std::size_t touched = 0;
    const std::size_t h0 = (std::size_t)L.plane_offset(-depth) * 8;
    for (std::size_t i = 0; i < whole.size(); ++i)
      if (i < h0 || i >= h0 + pb) touched += whole[i] != 0xEE;
    // all-reduce on one rank: max of u64 words and sum of doubles are identities
    unsigned long long hu[3] = {7ull, 0x7ff0000000000000ull, 3ull};
    double hd[2] = {1.5, -2.25};
    void* du = be->alloc(sizeof(hu));
    void* dd = be->alloc(sizeof(hd));
    be->copy(du, hu, sizeof(hu), CopyKind::H2D, kReduce);
    be->copy(dd, hd, sizeof(hd), CopyKind::H2D, kReduce);
    comm->allreduce(du, 3, RedType::U64, RedOp::Max, *be, kReduce);
    comm->allreduce(dd, 2, RedType::F64, RedOp::Sum, *be, kReduce);
    unsigned long long ru[3];
    double rd[2];
    be->copy(ru, du, sizeof(ru), CopyKind::D2H, kReduce);
    be->copy(rd, dd, sizeof(rd), CopyKind::D2H, kReduce);
    be->sync(kReduce);
    py::dict d;
    d["ok"] = ok;
    d["plane_bytes"] = pb;
    d["touched_outside"] = touched;
    d["allreduce_u64"] = py::make_tuple(ru[0], ru[1], ru[2]);
    d["allreduce_f64"] = py::make_tuple(rd[0], rd[1]);
    d["transport_ranks"] = comm->transport_ranks();
    d["name"] = std::string(comm->name());
    for (void* p : bufs) be->release(p);
    be->release(fa);
    be->release(fb);
    be->release(du);
    be->release(dd);
    comm.reset();
    return d;
  }, py::arg("device"), py::arg("sizes"), py::arg("n") = std::array<int64_t, 3>{6, 7, 9}, py::arg("depth") = 3);
  m.def("socket_listen", []() {
    int port = 0;
    int fd = net::listen_on("0.0.0.0", 0, &port);
    return py::make_tuple(fd, port);
  });
  m.def("usage", &Config::usage);
  m.def("config_parse", [](const std::vector<std::string>& args) {
    Config c = parse_args(args);
    py::dict d;
    d["n"] = py::make_tuple(c.n[0], c.n[1], c.n[2]);
    d["iter_max"] = c.iter_max;
    d["eps"] = c.eps;
    d["dtype"] = dtype_name(c.dtype);
    d["decomp"] = py::make_tuple(c.decomp[0], c.decomp[1], c.decomp[2]);
    d["virtual_ranks"] = c.virtual_ranks;
    d["use_graph"] = c.use_graph;
    d["overlap"] = c.overlap;
    d["check_every"] = c.check_every;
    d["kernel"] = c.kernel;
    d["output"] = c.output;
    d["compat"] = c.compat;
    d["banner"] = c.echo_banner();
    return d;
  });
  m.def("physics", [](int64_t nx, int64_t ny, int64_t nz) {
    Physics p = Physics::make(nx, ny, nz);
    py::dict d;
    d["h"] = py::make_tuple(p.h[0], p.h[1], p.h[2]);
    d["dt"] = p.dt;
    d["D"] = py::make_tuple(p.D[0], p.D[1], p.D[2]);
    return d;
  });
  m.def("dims_create", [](int n, std::array<int, 3> fixed) { return dims_create(n, fixed); },
        py::arg("nprocs"), py::arg("fixed") = std::array<int, 3>{0, 0, 0});
  m.def("decomposition", [](std::array<int64_t, 3> N, std::array<int, 3> dims) {
    int64_t n[3] = {N[0], N[1], N[2]};
    Decomposition d = Decomposition::make(n, dims);
    py::list out;
    for (auto& s : d.subs) out.append(sub_dict(s));
    return out;
  });
  m.def("split_interior", [](std::array<int64_t, 3> n, std::vector<int> neighbors) {
    Subdomain s;
    for (int a = 0; a < 3; ++a) s.n[a] = n[a];
    for (int f = 0; f < kNumFaces; ++f) s.neighbors[f] = neighbors.at(f);
    Box in;
    std::vector<Box> shell;
    Decomposition::split_interior(s, &in, &shell);
    auto tup = [](const Box& b) { return py::make_tuple(b.lo[0], b.hi[0], b.lo[1], b.hi[1], b.lo[2], b.hi[2]); };
    py::list sl;
    for (auto& b : shell) sl.append(tup(b));
    return py::make_tuple(tup(in), sl);
  });
  m.def("layout", [](std::array<int64_t, 3> n, int64_t esize, int64_t gx, int64_t gy, int64_t gz) {
          return layout_dict(to_layout(n, esize, gx, gy, gz));
        },
        py::arg("n"), py::arg("esize"), py::arg("gx") = 1, py::arg("gy") = 1, py::arg("gz") = 1);
  m.def("boundary_value", [](int64_t i, int64_t j, int64_t k, std::array<int64_t, 3> N, std::array<double, 3> h) {
    int64_t n[3] = {N[0], N[1], N[2]};
    double hh[3] = {h[0], h[1], h[2]};
    return boundary_value(i, j, k, n, hh);
  });
  m.attr("DEVICE_STATE_BYTES") = (int64_t)sizeof(DeviceState);
  m.attr("RESIDUAL_SLOTS") = (int64_t)kResidualSlots;
  m.attr("STATE_DONE_OFFSET") = (int64_t)offsetof(DeviceState, done);
  m.attr("RESIDUAL_INIT_BITS") = (unsigned long long)kResidualInitBits;

  // --- raw kernels (pointers as ints; stream = hipStream_t as int) ----------
  py::module_ hk = m.def_submodule("hip", "gfx950 kernels on device pointers");
  hk.def("stencil", [](const std::string& dt, int64_t in_ptr, int64_t out_ptr, std::array<int64_t, 3> n,
                       std::array<int64_t, 6> box, std::array<double, 3> D, int64_t state_ptr, int slot,
                       const std::string& kernel, int64_t stream) {
    DType t = dt_of(dt);
    auto p = sparams(in_ptr, out_ptr, n, (int64_t)dtype_size(t), box, D, state_ptr, slot);
    hip::stencil(t, p, KernelSpec::parse(kernel), reinterpret_cast<void*>(stream));
  });
  hk.def("stencil2", [](const std::string& dt, int64_t in_ptr, int64_t out_ptr, std::array<int64_t, 3> n,
                        std::array<double, 3> D, int64_t state_ptr, int slot, const std::string& kernel,
                        int64_t stream) {
    DType t = dt_of(dt);
    std::array<int64_t, 6> box = {0, n[0], 0, n[1], 0, n[2]};
    auto p = sparams(in_ptr, out_ptr, n, (int64_t)dtype_size(t), box, D, state_ptr, slot);
    KernelSpec k = KernelSpec::parse(kernel);
    if (!k.multi_step()) {  // two steps: the lean kernel at K = 2
      k.kind = KernelSpec::TBL;
      k.K = 2;
    }
    hip::sweep(t, p, k, reinterpret_cast<void*>(stream));
  });
  // multi-step sweep on a sub-box of a layout with gx ghost planes, u range ux
  // (the solver's slab path); kernel = tl2..tl6 spec
  hk.def("stencil_sweep", [](const std::string& dt, int64_t in_ptr, int64_t out_ptr, std::array<int64_t, 3> n,
                             int64_t gx, std::array<int64_t, 6> box, std::array<int64_t, 2> ux,
                             std::array<double, 3> D, int64_t state_ptr, int slot, const std::string& kernel,
                             int64_t stream) {
    DType t = dt_of(dt);
    auto p = sparams(in_ptr, out_ptr, n, (int64_t)dtype_size(t), box, D, state_ptr, slot);
    p.L = to_layout(n, (int64_t)dtype_size(t), gx);
    p.ux[0] = ux[0];
    p.ux[1] = ux[1];
    KernelSpec k = KernelSpec::parse(kernel);
    if (!k.multi_step()) throw UsageError("stencil_sweep needs a tl2..tl6 kernel");
    hip::sweep(t, p, k, reinterpret_cast<void*>(stream));
  });
  // deep ghosts on every axis (block decompositions): g = (gx, gy, gz),
  // u = update ranges (ux0, ux1, uy0, uy1, uz0, uz1)
  hk.def("stencil_sweep3", [](const std::string& dt, int64_t in_ptr, int64_t out_ptr, std::array<int64_t, 3> n,
                              std::array<int64_t, 3> g, std::array<int64_t, 6> box, std::array<int64_t, 6> u,
                              std::array<double, 3> D, int64_t state_ptr, int slot, const std::string& kernel,
                              int64_t stream) {
    DType t = dt_of(dt);
    auto p = sparams(in_ptr, out_ptr, n, (int64_t)dtype_size(t), box, D, state_ptr, slot);
    p.L = to_layout(n, (int64_t)dtype_size(t), g[0], g[1], g[2]);
    for (int e = 0; e < 2; ++e) {
      p.ux[e] = u[e];
      p.uy[e] = u[2 + e];
      p.uz[e] = u[4 + e];
    }
    KernelSpec k = KernelSpec::parse(kernel);
    if (!k.multi_step()) throw UsageError("stencil_sweep3 needs a tl2..tl6 kernel");
    hip::sweep(t, p, k, reinterpret_cast<void*>(stream));
  });
  hk.def("init_field", [](const std::string& dt, int64_t ptr, std::array<int64_t, 3> n, std::array<int64_t, 3> gstart,
                          std::array<int64_t, 3> N, std::array<double, 3> h, int64_t stream) {
    DType t = dt_of(dt);
    InitParams p;
    p.field = reinterpret_cast<void*>(ptr);
    p.L = to_layout(n, (int64_t)dtype_size(t));
    for (int a = 0; a < 3; ++a) {
      p.gstart[a] = gstart[a];
      p.N[a] = N[a];
      p.h[a] = h[a];
    }
    hip::init_field(t, p, reinterpret_cast<void*>(stream));
  });
  hk.def("pack_box", [](const std::string& dt, int64_t f, std::array<int64_t, 3> n, std::array<int64_t, 6> box,
                        int64_t buf, int64_t stream) {
    DType t = dt_of(dt);
    hip::pack_box(t, reinterpret_cast<void*>(f), to_layout(n, (int64_t)dtype_size(t)), to_box(box),
                  reinterpret_cast<void*>(buf), reinterpret_cast<void*>(stream));
  });
  hk.def("unpack_box", [](const std::string& dt, int64_t f, std::array<int64_t, 3> n, std::array<int64_t, 6> box,
                          int64_t buf, int64_t stream) {
    DType t = dt_of(dt);
    hip::unpack_box(t, reinterpret_cast<void*>(f), to_layout(n, (int64_t)dtype_size(t)), to_box(box),
                    reinterpret_cast<void*>(buf), reinterpret_cast<void*>(stream));
  });
  hk.def("bandwidth_probe", [](int kind, int64_t src, int64_t dst, int64_t bytes, int blocks, int64_t stream) {
    hip::bandwidth_probe(kind, reinterpret_cast<const void*>(src), reinterpret_cast<void*>(dst), bytes, blocks,
                         reinterpret_cast<void*>(stream));
  });
  hk.def("check_convergence", [](int64_t state_ptr, int slot, int64_t stream) {
    hip::check_convergence(reinterpret_cast<DeviceState*>(state_ptr), slot, reinterpret_cast<void*>(stream));
  });

  py::module_ ck = m.def_submodule("cpu", "OpenMP host kernels on host pointers");
  ck.def("stencil", [](const std::string& dt, int64_t in_ptr, int64_t out_ptr, std::array<int64_t, 3> n,
                       std::array<int64_t, 6> box, std::array<double, 3> D, int64_t state_ptr, int slot) {
    DType t = dt_of(dt);
    auto p = sparams(in_ptr, out_ptr, n, (int64_t)dtype_size(t), box, D, state_ptr, slot);
    py::gil_scoped_release nogil;
    cpu::stencil(t, p);
  });
  ck.def("stencil_sweep", [](const std::string& dt, int64_t in_ptr, int64_t out_ptr, std::array<int64_t, 3> n,
                             int64_t gx, std::array<int64_t, 6> box, std::array<int64_t, 2> ux,
                             std::array<double, 3> D, int64_t state_ptr, int slot, const std::string& kernel) {
    DType t = dt_of(dt);
    auto p = sparams(in_ptr, out_ptr, n, (int64_t)dtype_size(t), box, D, state_ptr, slot);
    p.L = to_layout(n, (int64_t)dtype_size(t), gx);
    p.ux[0] = ux[0];
    p.ux[1] = ux[1];
    KernelSpec k = KernelSpec::parse(kernel);
    if (!k.multi_step()) throw UsageError("stencil_sweep needs a tl2..tl6 kernel");
    std::vector<char> s0(p.L.bytes()), s1(p.L.bytes());
    py::gil_scoped_release nogil;
    cpu::stencil_multi(t, p, k.K, s0.data(), s1.data());
  });
  ck.def("stencil_sweep3", [](const std::string& dt, int64_t in_ptr, int64_t out_ptr, std::array<int64_t, 3> n,
                              std::array<int64_t, 3> g, std::array<int64_t, 6> box, std::array<int64_t, 6> u,
                              std::array<double, 3> D, int64_t state_ptr, int slot, const std::string& kernel) {
    DType t = dt_of(dt);
    auto p = sparams(in_ptr, out_ptr, n, (int64_t)dtype_size(t), box, D, state_ptr, slot);
    p.L = to_layout(n, (int64_t)dtype_size(t), g[0], g[1], g[2]);
    for (int e = 0; e < 2; ++e) {
      p.ux[e] = u[e];
      p.uy[e] = u[2 + e];
      p.uz[e] = u[4 + e];
    }
    KernelSpec k = KernelSpec::parse(kernel);
    if (!k.multi_step()) throw UsageError("stencil_sweep3 needs a tl2..tl6 kernel");
    std::vector<char> s0(p.L.bytes()), s1(p.L.bytes());
    py::gil_scoped_release nogil;
    cpu::stencil_multi(t, p, k.K, s0.data(), s1.data());
  });
  ck.def("init_field", [](const std::string& dt, int64_t ptr, std::array<int64_t, 3> n, std::array<int64_t, 3> gstart,
                          std::array<int64_t, 3> N, std::array<double, 3> h) {
    DType t = dt_of(dt);
    InitParams p;
    p.field = reinterpret_cast<void*>(ptr);
    p.L = to_layout(n, (int64_t)dtype_size(t));
    for (int a = 0; a < 3; ++a) {
      p.gstart[a] = gstart[a];
      p.N[a] = N[a];
      p.h[a] = h[a];
    }
    cpu::init_field(t, p);
  });

  // --- solver ---------------------------------------------------------------
  py::class_<ReferenceScheme>(m, "ReferenceScheme",
                              "The reference's shared-plane decomposition scheme, all ranks in-process (CPU)")
      .def(py::init([](std::array<int64_t, 3> N, std::array<int, 3> dims) {
             int64_t n[3] = {N[0], N[1], N[2]};
             return new ReferenceScheme(n, dims);
           }),
           py::arg("N"), py::arg("dims"))
      .def_property_readonly("chunk", [](const ReferenceScheme& r) { return r.chunk(); })
      .def_property_readonly("ranks", &ReferenceScheme::ranks)
      .def("run", [](ReferenceScheme& rs, int64_t iter_max, double eps) {
             ReferenceSchemeResult r;
             {
               py::gil_scoped_release nogil;
               r = rs.run(iter_max, eps);
             }
             py::dict d;
             d["converged"] = r.converged;
             d["conv_iter"] = r.conv_iter;
             d["iterations"] = r.iterations;
             d["seconds"] = r.seconds;
             d["norm_rank0"] = r.norm_rank0;
             d["error_percent_rank0"] = 100.0 * r.error_rank0;
             d["error_percent_global"] = 100.0 * r.error_global;
             d["last_residual_rank0"] = r.last_residual_rank0;
             return d;
           },
           py::arg("iter_max"), py::arg("eps"))
      .def("gather", [](const ReferenceScheme& rs) {
        auto g = rs.gather();
        return py::array_t<double>(g.size(), g.data());
      })
      .def("write_tecplot", &ReferenceScheme::write_tecplot);

  py::class_<Solver>(m, "Solver")
      .def(py::init(&create_solver), py::arg("args"), py::arg("rank") = 0, py::arg("size") = 1,
           py::arg("comm") = "local", py::arg("unique_id") = py::bytes(), py::arg("listen_fd") = -1,
           py::arg("addrs") = std::vector<std::string>{}, py::arg("device") = -1)
      .def("initialize", [](Solver& s) {
        py::gil_scoped_release nogil;
        s.initialize();
      })
      .def("run", [](Solver& s) {
        RunResult r;
        {
          py::gil_scoped_release nogil;
          r = s.run();
        }
        py::dict d;
        d["converged"] = r.converged;
        d["fault"] = r.fault;
        d["conv_iter"] = r.conv_iter;
        d["iterations"] = r.iterations;
        d["issued"] = r.issued;
        d["seconds"] = r.seconds;
        d["norm"] = r.norm;
        d["last_residual"] = r.last_residual;
        d["glups"] = r.glups;
        return d;
      })
      .def("step", [](Solver& s, int64_t n) {
        py::gil_scoped_release nogil;
        s.step(n);
      })
      .def("synchronize", [](Solver& s) {
        py::gil_scoped_release nogil;
        s.synchronize();
      })
      .def("prepare_steps", [](Solver& s, int64_t n) {
        py::gil_scoped_release nogil;
        s.prepare_steps(n);
      })
      .def("preheat", [](Solver& s, int sweeps) {
        py::gil_scoped_release nogil;
        return s.preheat(sweeps);
      })
      .def("state", [](Solver& s) {
        HostState h = s.state();
        py::dict d;
        d["norm"] = h.norm;
        d["eps"] = h.eps;
        d["last_residual"] = h.last_residual;
        d["iter"] = h.iter;
        d["conv_iter"] = h.conv_iter;
        d["done"] = h.done;
        d["fault"] = h.fault;
        return d;
      })
      .def("compute_error", [](Solver& s) {
        double g = 0, l = 0;
        s.compute_error(&g, &l);
        return py::make_tuple(g, l);
      })
      .def("gather_global", [](Solver& s) -> py::object {
        std::vector<double> v;
        bool root;
        {
          py::gil_scoped_release nogil;
          root = s.gather_global(&v);
        }
        if (!root) return py::none();
        const auto& N = s.decomposition().N;
        return to_numpy(std::move(v), {(py::ssize_t)N[0], (py::ssize_t)N[1], (py::ssize_t)N[2]});
      })
      .def("local_field", [](Solver& s, int idx, bool ghosts) {
        auto v = s.local_field(idx, ghosts);
        const auto& sd = s.local_subdomain(idx);
        const int g = ghosts ? 2 : 0;
        return to_numpy(std::move(v), {(py::ssize_t)(sd.n[0] + g), (py::ssize_t)(sd.n[1] + g), (py::ssize_t)(sd.n[2] + g)});
      }, py::arg("idx") = 0, py::arg("ghosts") = false)
      .def("local_subdomain", [](Solver& s, int i) { return sub_dict(s.local_subdomain(i)); })
      .def("local_layout", [](Solver& s, int i) { return layout_dict(s.local_layout(i)); })
      .def("local_field_ptr", [](Solver& s, int i) { return reinterpret_cast<int64_t>(s.local_field_ptr(i)); })
      .def("write_tecplot", [](Solver& s, const std::string& path, const std::string& layout) {
        py::gil_scoped_release nogil;
        s.write_tecplot(path, layout);
      }, py::arg("path"), py::arg("layout") = "auto")
      .def("save_checkpoint", [](Solver& s, const std::string& d) {
        py::gil_scoped_release nogil;
        s.save_checkpoint(d);
      })
      .def("load_checkpoint", [](Solver& s, const std::string& d) {
        py::gil_scoped_release nogil;
        s.load_checkpoint(d);
      })
      .def("inject", &Solver::inject, py::arg("idx"), py::arg("i"), py::arg("j"), py::arg("k"),
           py::arg("value"), py::arg("previous") = false)
      .def("verify_halos", [](Solver& s) {
        py::gil_scoped_release nogil;
        return s.verify_halos();
      })
      .def("link_probe", [](Solver& s, std::size_t bytes, int reps) {
        py::gil_scoped_release nogil;
        return s.link_probe(bytes, reps);
      }, py::arg("bytes"), py::arg("reps") = 5)
      .def("set_phase_timing", &Solver::set_phase_timing)
      .def("phase_times", &Solver::phase_times)
      .def("profile_sweeps", [](Solver& s, int n) {
        std::vector<std::pair<std::string, double>> v;
        {
          py::gil_scoped_release nogil;
          v = s.profile_sweeps(n);
        }
        py::dict d;
        for (auto& kv : v) d[py::str(kv.first)] = kv.second;
        return d;
      }, py::arg("n") = 8)
      .def_property_readonly("num_local", &Solver::num_local)
      .def_property_readonly("is_root", &Solver::is_root)
      .def_property_readonly("process_rank", &Solver::process_rank)
      .def_property_readonly("interior_points", &Solver::interior_points)
      .def_property_readonly("iterations_issued", &Solver::iterations_issued)
      .def_property_readonly("graph_launches", &Solver::graph_launches)
      .def_property_readonly("stream_graphs_state", &Solver::stream_graphs_state)
      .def_property_readonly("stream_graphs_note", &Solver::stream_graphs_note)
      .def_property_readonly("ranks_per_device", &Solver::ranks_per_device)
      .def_property_readonly("monotone_check", &Solver::monotone_check)
      .def_property_readonly("comm_transport_ranks", [](Solver& s) { return s.comm().transport_ranks(); })
      .def_property_readonly("device", [](Solver& s) { return s.backend().device(); })
      .def_property_readonly("reserved_cus", [](Solver& s) { return s.backend().reserved_cus(); })
      .def_property_readonly("planned_bytes", &Solver::planned_bytes)
      .def_property_readonly("mem_free_before", &Solver::mem_free_before)
      .def_property_readonly("mem_total", &Solver::mem_total)
      // (free, total) bytes of the backend's memory now (HBM: hipMemGetInfo)
      .def("mem_info", [](Solver& s) -> py::tuple {
        std::size_t f = 0, t = 0;
        if (!s.backend().mem_info(&f, &t)) return py::make_tuple(py::none(), py::none());
        return py::make_tuple(f, t);
      })
      .def_property_readonly("kernel_name", &Solver::kernel_name)
      .def_property_readonly("temporal_blocking", &Solver::temporal_blocking)
      .def_property_readonly("temporal_steps", &Solver::temporal_steps)
      .def_property_readonly("field_buffers", &Solver::field_buffers)
      .def_property_readonly("ghost_depth", &Solver::ghost_depth)
      .def_property_readonly("long_halo_sweeps", &Solver::long_halo_sweeps)
      .def("sweep_pieces", &Solver::sweep_pieces, py::arg("local") = 0)
      .def_property_readonly("long_major", &Solver::long_major)
      .def_property_readonly("long_remainders",
                             [](const Solver& s) {
                               std::vector<int> r;
                               for (int i = 1; i < s.temporal_steps(); ++i)
                                 if ((s.long_remainders() >> i) & 1u) r.push_back(i);
                               return r;
                             })
      .def_property_readonly("sweep_costs",
                             [](const Solver& s) {
                               py::dict d;
                               for (auto& kv : s.sweep_costs()) d[py::str(kv.first)] = kv.second;
                               return d;
                             })
      .def_property_readonly("backend_name", [](Solver& s) { return std::string(s.backend().name()); })
      .def_property_readonly("comm_name", [](Solver& s) { return std::string(s.comm().name()); })
      .def_property_readonly("rccl_p2p_channels", [](Solver&) { return rccl_p2p_channels_env(); })
      .def_property_readonly("comm_size", [](Solver& s) { return s.comm().size(); })
      .def_property_readonly("dims", [](Solver& s) { return s.decomposition().topo.dims; })
      .def_property_readonly("physics", [](Solver& s) {
        const Physics& p = s.physics();
        py::dict d;
        d["h"] = py::make_tuple(p.h[0], p.h[1], p.h[2]);
        d["dt"] = p.dt;
        d["D"] = py::make_tuple(p.D[0], p.D[1], p.D[2]);
        return d;
      });
}
