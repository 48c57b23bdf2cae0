// pybind11 module `_cek`: the single Python↔C++ boundary of the runtime.
// Every compute() crosses it once and releases the GIL for the fan-out.
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "balancer.h"
#include "copy_engine.h"
#include "cores.h"
#include "device.h"
#include "dist.h"
#include "jit.h"
#include "memory.h"
#include "pool.h"
#include "probe.h"
#include "refloops.h"
#include "xgmi.h"

namespace py = pybind11;
using namespace cek;

namespace {

class PyExchanger : public Exchanger {
 public:
  using Exchanger::Exchanger;
  std::vector<double> allgather(const std::vector<double>& local) override {
    PYBIND11_OVERRIDE_PURE(std::vector<double>, Exchanger, allgather, local);
  }
  int rank() const override { PYBIND11_OVERRIDE_PURE(int, Exchanger, rank, ); }
  int world() const override { PYBIND11_OVERRIDE_PURE(int, Exchanger, world, ); }
};

// A data plane implemented in Python (e.g. torch.distributed gloo over host
// memory for CPU devices): pointers and streams cross as integers.  Called
// from compute() with the GIL released, so every override re-acquires it.
class PyComm : public Comm {
 public:
  int rank() const override { PYBIND11_OVERRIDE_PURE(int, Comm, rank, ); }
  int world() const override { PYBIND11_OVERRIDE_PURE(int, Comm, world, ); }
  void broadcast(void* dptr, uint64_t bytes, int root, hipStream_t s) override {
    call("broadcast", reinterpret_cast<uint64_t>(dptr), bytes, root, reinterpret_cast<uint64_t>(s));
  }
  void allgatherv(void* dptr, const std::vector<uint64_t>& offsets, const std::vector<uint64_t>& sizes,
                  hipStream_t s) override {
    call("allgatherv", reinterpret_cast<uint64_t>(dptr), offsets, sizes, reinterpret_cast<uint64_t>(s));
  }
  void allreduce_sum_f32(void* dptr, uint64_t count, hipStream_t s) override {
    call("allreduce_sum_f32", reinterpret_cast<uint64_t>(dptr), count, reinterpret_cast<uint64_t>(s));
  }
  void allreduce_sum_f64(void* dptr, uint64_t count, hipStream_t s) override {
    call("allreduce_sum_f64", reinterpret_cast<uint64_t>(dptr), count, reinterpret_cast<uint64_t>(s));
  }

 private:
  template <typename... A>
  void call(const char* name, A&&... args) {
    py::gil_scoped_acquire g;
    py::function f = py::get_override(static_cast<const Comm*>(this), name);
    if (!f) throw Error(std::string("Comm.") + name + " is not implemented by this communicator");
    f(std::forward<A>(args)...);
  }
};

uint64_t py_host_alloc(uint64_t bytes, uint64_t align) {
  bool pinned = false;
  return reinterpret_cast<uint64_t>(host_alloc(bytes, align, &pinned));
}

}  // namespace

PYBIND11_MODULE(_cek, m) {
  m.doc() = "cekirdekler_amd native runtime (HIP/gfx950)";

  py::register_exception<Error>(m, "CekError", PyExc_RuntimeError);

  py::enum_<DevType>(m, "DevType")
      .value("CPU", kCPU)
      .value("GPU", kGPU)
      .value("ACC", kACC)
      .export_values();

  py::class_<DeviceInfo>(m, "DeviceInfo")
      .def(py::init<>())
      .def_readwrite("type", &DeviceInfo::type)
      .def_readwrite("ordinal", &DeviceInfo::ordinal)
      .def_readwrite("name", &DeviceInfo::name)
      .def_readwrite("arch", &DeviceInfo::arch)
      .def_readwrite("vendor", &DeviceInfo::vendor)
      .def_readwrite("platform", &DeviceInfo::platform)
      .def_readwrite("compute_units", &DeviceInfo::compute_units)
      .def_readwrite("mem_bytes", &DeviceInfo::mem_bytes)
      .def_readwrite("dedicated_memory", &DeviceInfo::dedicated_memory)
      .def_readwrite("streaming", &DeviceInfo::streaming)
      .def_readwrite("cpu_threads", &DeviceInfo::cpu_threads)
      .def_readwrite("pci_bus", &DeviceInfo::pci_bus)
      .def_readwrite("pci_device", &DeviceInfo::pci_device)
      .def_readwrite("clock_khz", &DeviceInfo::clock_khz)
      .def_readwrite("lds_per_block", &DeviceInfo::lds_per_block)
      .def_readwrite("cu_part", &DeviceInfo::cu_part)
      .def_readwrite("cu_parts", &DeviceInfo::cu_parts)
      .def("describe", &DeviceInfo::describe)
      .def("__repr__", [](const DeviceInfo& d) { return "<DeviceInfo " + d.describe() + ">"; });

  m.def("partition_cus", &partition_cus, py::arg("ncu"), py::arg("parts"), py::arg("p"));
  m.def("gpu_count", &gpu_count);
  m.def("enumerate_devices", &enumerate_devices);
  m.def("gpu_info", &gpu_info);
  m.def("cpu_info", &cpu_info, py::arg("threads") = -1);
  m.def("enable_peer_access", &enable_peer_access);
  m.def("enable_peer_access_among", &enable_peer_access_among, py::arg("ordinals"));
  m.def("peer_path", &peer_path, py::arg("matrix"));
  // query only (no context is created, nothing is enabled): hipDeviceCanAccessPeer
  // between every pair of visible GPUs
  m.def("can_access_peer_matrix", []() {
    const int n = gpu_count();
    std::vector<std::vector<int>> m(n, std::vector<int>(n, 1));
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        if (i == j) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, i, j) != hipSuccess) {
          (void)hipGetLastError();
          can = 0;
        }
        m[i][j] = can;
      }
    return m;
  });

  py::class_<KernelSig>(m, "KernelSig")
      .def_readonly("name", &KernelSig::name)
      .def_readonly("arity", &KernelSig::arity)
      .def("__repr__", [](const KernelSig& k) { return "<Kernel " + k.name + "/" + std::to_string(k.arity) + ">"; });
  m.def("parse_kernels", &parse_kernels);
  m.def("is_opencl_dialect", &is_opencl_dialect);
  m.def("gpu_rewrite", &gpu_rewrite);
  m.def("now_ms", &now_ms, "the runtime's host clock (steady clock, ms): the clock of every timeline");
  m.def("cpu_rewrite", &cpu_rewrite);
  m.def("cache_dir", &cache_dir);
  m.def("hash_hex", &hash_hex);
  m.def("compile_gpu", [](const std::string& src, const std::vector<std::string>& opts, const std::string& arch) {
    std::string code, log;
    bool ok = compile_gpu(gpu_rewrite(src), opts, arch, code, log);
    return py::make_tuple(ok, py::bytes(code), log);
  }, py::arg("src"), py::arg("options") = std::vector<std::string>{}, py::arg("arch") = "gfx950");

  m.def("host_alloc", &py_host_alloc, py::arg("bytes"), py::arg("align") = 4096);
  m.def("host_free", [](uint64_t p) { host_free(reinterpret_cast<void*>(p)); });
  m.def("host_is_pinned", [](uint64_t p) { return host_is_pinned(reinterpret_cast<void*>(p)); });
  m.def("host_register", [](uint64_t p, uint64_t n) { return host_register(reinterpret_cast<void*>(p), n); });
  m.def("host_unregister", [](uint64_t p) { host_unregister(reinterpret_cast<void*>(p)); });
  // Unified-address copy between any two of {host, GPU i, GPU j}: device→device
  // goes over xGMI (peer), host↔device over PCIe; plain memcpy without a GPU.
  m.def("memcpy_default", [](uint64_t d, uint64_t s, uint64_t n) {
    py::gil_scoped_release r;
    if (n == 0) return;
    if (gpu_count() == 0) {
      copy_memory(reinterpret_cast<void*>(d), reinterpret_cast<const void*>(s), n);
      return;
    }
    CEK_HIP(hipMemcpy(reinterpret_cast<void*>(d), reinterpret_cast<const void*>(s), n, hipMemcpyDefault));
  });
  py::class_<CopyEngine>(m, "CopyEngine")
      .def(py::init<>())
      .def("copy", [](CopyEngine& e, uint64_t d, int dd, uint64_t s, int sd, uint64_t n) {
        e.copy(reinterpret_cast<void*>(d), dd, reinterpret_cast<const void*>(s), sd, n);
      }, py::arg("dst"), py::arg("dst_dev"), py::arg("src"), py::arg("src_dev"), py::arg("bytes"),
         py::call_guard<py::gil_scoped_release>())
      .def("sync", &CopyEngine::sync, py::call_guard<py::gil_scoped_release>())
      .def("reset_counters", &CopyEngine::reset_counters)
      .def_readonly("p2p_bytes", &CopyEngine::p2p_bytes)
      .def_readonly("h2d_bytes", &CopyEngine::h2d_bytes)
      .def_readonly("d2h_bytes", &CopyEngine::d2h_bytes)
      .def_readonly("host_bytes", &CopyEngine::host_bytes)
      .def_readonly("copies", &CopyEngine::copies)
      .def_readwrite("record_timeline", &CopyEngine::record_timeline)
      .def("timeline", [](CopyEngine& e) {
        std::vector<CopyEngine::Span> spans;
        {
          py::gil_scoped_release nogil;
          spans = e.timeline();
        }
        py::list out;
        for (auto& s : spans) {
          py::dict d;
          d["device"] = s.ordinal;
          d["kind"] = s.kind;
          d["bytes"] = s.bytes;
          d["abs_begin_ms"] = s.abs_begin_ms;
          d["abs_end_ms"] = s.abs_end_ms;
          out.append(d);
        }
        return out;
      });
  m.def("device_synchronize", [](int ordinal) {
    py::gil_scoped_release r;
    if (gpu_count() == 0) return;
    CEK_HIP(hipSetDevice(ordinal));
    CEK_HIP(hipDeviceSynchronize());
  });
  m.def("copy_memory", [](uint64_t d, uint64_t s, uint64_t n) {
    py::gil_scoped_release r;
    copy_memory(reinterpret_cast<void*>(d), reinterpret_cast<const void*>(s), n);
  });

  m.def("wave_reference_scalar", [](uint64_t base, uint64_t normals, uint64_t out, long long n, float ctr, float t) {
    py::gil_scoped_release r;
    wave_reference_scalar(reinterpret_cast<const float*>(base), reinterpret_cast<const float*>(normals),
                          reinterpret_cast<float*>(out), n, ctr, t);
  }, "the reference wave example's single-threaded scalar CPU loop (Kamera.cs:208-218); pointers to packed xyz floats");

  m.def("load_balance", [](std::vector<double> bench, bool smooth, std::vector<std::vector<double>> history,
                           long long total, std::vector<long long> ranges, long long step) {
    load_balance(bench, smooth, history, total, ranges, step);
    return py::make_tuple(ranges, history);
  });
  m.def("predict_split", [](std::vector<double> bench, double wall, long long total, std::vector<long long> ranges,
                            long long step, py::object state, bool warm) {
    // pure form for tests: `state` is a FitState
    auto* fs = state.cast<FitState*>();
    bool ok = predict_split(*fs, bench, wall, total, ranges, step, warm);
    return py::make_tuple(ok, ranges, fs->decision);
  }, py::arg("bench"), py::arg("wall"), py::arg("total"), py::arg("ranges"), py::arg("step"), py::arg("state"),
     py::arg("warm") = true);
  py::class_<FitState>(m, "FitState")
      .def(py::init<>())
      .def_readonly("decision", &FitState::decision)
      .def_readonly("a", &FitState::a)
      .def_readonly("b", &FitState::b)
      .def_readonly("o_multi", &FitState::o_multi)
      .def_readonly("single_wall", &FitState::single_wall)
      .def_readonly("predicted_multi_ms", &FitState::predicted_multi_ms)
      .def_readonly("multi_wall", &FitState::multi_wall)
      .def_readonly("law_wall", &FitState::law_wall);
  m.def("initial_split", [](int devices, bool smooth, std::vector<std::vector<double>> history,
                            long long total, long long step) {
    std::vector<long long> ranges;
    initial_split(devices, smooth, history, total, ranges, step);
    return py::make_tuple(ranges, history);
  });
  m.attr("HISTORY_DEPTH") = kHistoryDepth;

  py::class_<ArraySpec>(m, "ArraySpec")
      .def(py::init<>())
      .def(py::init([](uint64_t uid, uint64_t host, uint64_t bytes, int elem_size, bool read, bool partial,
                       bool write, bool write_all, bool ro, bool wo, bool zc, int epw, int epg, bool gather) {
             ArraySpec a;
             a.uid = uid;
             a.host = reinterpret_cast<void*>(host);
             a.bytes = bytes;
             a.elem_size = elem_size;
             a.read = read;
             a.partial = partial;
             a.write = write;
             a.write_all = write_all;
             a.ro = ro;
             a.wo = wo;
             a.zc = zc;
             a.epw = epw;
             a.epg = epg;
             a.gather = gather;
             return a;
           }),
           py::arg("uid"), py::arg("host"), py::arg("bytes"), py::arg("elem_size"), py::arg("read") = true,
           py::arg("partial") = false, py::arg("write") = true, py::arg("write_all") = false,
           py::arg("ro") = false, py::arg("wo") = false, py::arg("zc") = false, py::arg("epw") = 1, py::arg("epg") = 0,
           py::arg("gather") = false)
      .def_readwrite("uid", &ArraySpec::uid)
      .def_property("host", [](const ArraySpec& a) { return reinterpret_cast<uint64_t>(a.host); },
                    [](ArraySpec& a, uint64_t p) { a.host = reinterpret_cast<void*>(p); })
      .def_readwrite("bytes", &ArraySpec::bytes)
      .def_readwrite("elem_size", &ArraySpec::elem_size)
      .def_readwrite("read", &ArraySpec::read)
      .def_readwrite("partial", &ArraySpec::partial)
      .def_readwrite("write", &ArraySpec::write)
      .def_readwrite("write_all", &ArraySpec::write_all)
      .def_readwrite("ro", &ArraySpec::ro)
      .def_readwrite("wo", &ArraySpec::wo)
      .def_readwrite("zc", &ArraySpec::zc)
      .def_readwrite("epw", &ArraySpec::epw)
      .def_readwrite("epg", &ArraySpec::epg)
      .def_readwrite("gather", &ArraySpec::gather)
      .def_readwrite("blob_begin", &ArraySpec::blob_begin)
      .def_readwrite("blob_count", &ArraySpec::blob_count);

  py::class_<ComputeCall>(m, "ComputeCall")
      .def(py::init<>())
      .def_readwrite("kernels", &ComputeCall::kernels)
      .def_readwrite("repeats", &ComputeCall::repeats)
      .def_readwrite("repeat_kernel", &ComputeCall::repeat_kernel)
      .def_readwrite("arrays", &ComputeCall::arrays)
      .def_readwrite("global_range", &ComputeCall::global_range)
      .def_readwrite("local_range", &ComputeCall::local_range)
      .def_readwrite("global_offset", &ComputeCall::global_offset)
      .def_readwrite("compute_id", &ComputeCall::compute_id)
      .def_readwrite("pipeline", &ComputeCall::pipeline)
      .def_readwrite("pipeline_event", &ComputeCall::pipeline_event)
      .def_readwrite("blobs", &ComputeCall::blobs)
      .def_readwrite("granularity", &ComputeCall::granularity)
      .def_readwrite("blob_bounds", &ComputeCall::blob_bounds);

  py::class_<CoresConfig>(m, "CoresConfig")
      .def(py::init<>())
      .def_readwrite("queue_concurrency", &CoresConfig::queue_concurrency)
      .def_readwrite("no_pipelining", &CoresConfig::no_pipelining)
      .def_readwrite("smooth", &CoresConfig::smooth)
      .def_readwrite("options", &CoresConfig::options)
      .def_readwrite("prebuilt", &CoresConfig::prebuilt);

  py::class_<ComputeRecord>(m, "ComputeRecord")
      .def_readonly("compute_id", &ComputeRecord::compute_id)
      .def_readonly("wall_ms", &ComputeRecord::wall_ms)
      .def_readonly("ranges", &ComputeRecord::ranges)
      .def_readonly("references", &ComputeRecord::references)
      .def_readonly("device_ms", &ComputeRecord::device_ms)
      .def_readonly("h2d_bytes", &ComputeRecord::h2d_bytes)
      .def_readonly("d2h_bytes", &ComputeRecord::d2h_bytes)
      .def_readonly("p2p_bytes", &ComputeRecord::p2p_bytes)
      .def_readonly("gather_bytes", &ComputeRecord::gather_bytes)
      .def_readonly("staged_bytes", &ComputeRecord::staged_bytes)
      .def_readonly("p2p_path", &ComputeRecord::p2p_path)
      .def_readonly("pipelined", &ComputeRecord::pipelined);

  py::class_<Exchanger, PyExchanger, std::shared_ptr<Exchanger>>(m, "Exchanger")
      .def(py::init<>())
      .def("allgather", &Exchanger::allgather)
      .def("rank", &Exchanger::rank)
      .def("world", &Exchanger::world);

  py::class_<ShmExchanger, Exchanger, std::shared_ptr<ShmExchanger>>(m, "ShmExchanger")
      .def(py::init<const std::string&, int, int, int, double>(), py::arg("name"), py::arg("rank"),
           py::arg("world"), py::arg("max_values") = 64, py::arg("timeout_s") = 300.0)
      .def("allgather", &ShmExchanger::allgather, py::call_guard<py::gil_scoped_release>())
      .def("unlink", &ShmExchanger::unlink);

  py::class_<Comm, PyComm, std::shared_ptr<Comm>>(m, "Comm")
      .def(py::init<>())
      .def("rank", &Comm::rank)
      .def("world", &Comm::world);

  py::class_<RcclComm, Comm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def(py::init([](py::bytes uid, int rank, int world, int device) {
        // copy the id while holding the GIL; only the RCCL rendezvous runs
        // without it (the bytes object is released by pybind11, GIL held)
        std::string id(uid);
        py::gil_scoped_release r;
        return std::make_shared<RcclComm>(id, rank, world, device);
      }))
      .def("broadcast", [](RcclComm& c, uint64_t p, uint64_t bytes, int root, uint64_t stream) {
        c.broadcast(reinterpret_cast<void*>(p), bytes, root, reinterpret_cast<hipStream_t>(stream));
      }, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_sum_f32", [](RcclComm& c, uint64_t p, uint64_t n, uint64_t stream) {
        c.allreduce_sum_f32(reinterpret_cast<void*>(p), n, reinterpret_cast<hipStream_t>(stream));
      }, py::call_guard<py::gil_scoped_release>());

  m.def("launch_rate_probe", [](int ordinal, const std::string& co, const std::string& kernel, int threads,
                                int launches, int mode) {
        LaunchRate r;
        {
          py::gil_scoped_release rel;
          r = launch_rate_probe(ordinal, co, kernel, threads, launches, mode);
        }
        py::dict d;
        d["threads"] = r.threads;
        d["launches_per_thread"] = r.launches;
        d["host_ms"] = r.host_ms;
        d["drain_ms"] = r.drain_ms;
        d["launches_per_s"] = r.launches_per_s;
        d["per_thread_ms"] = r.per_thread_ms;
        return d;
      }, py::arg("ordinal"), py::arg("code_object"), py::arg("kernel"), py::arg("threads"), py::arg("launches"),
      py::arg("mode") = 0);

  m.def("allgatherv_plan", [](int rank, int world, const std::vector<uint64_t>& offsets,
                              const std::vector<uint64_t>& sizes) {
        py::list out;
        for (const auto& op : allgatherv_plan(rank, world, offsets, sizes))
          out.append(py::make_tuple(op.send ? "send" : "recv", op.peer, op.offset, op.bytes));
        return out;
      }, py::arg("rank"), py::arg("world"), py::arg("offsets"), py::arg("sizes"),
      "The (kind, peer, offset, bytes) point-to-point ops one rank issues for an uneven all-gather-v.");

  // device→device copy engines (xgmi.h)
  m.def("measure_copy", [](int src, int dst, uint64_t bytes, int engine, int reps, int stream_ordinal) {
        CopyMeasure r;
        {
          py::gil_scoped_release rel;
          r = measure_copy(src, dst, bytes, engine, reps, stream_ordinal);
        }
        py::dict d;
        d["src"] = r.src;
        d["dst"] = r.dst;
        d["engine"] = r.engine == kCopyKernel ? "kernel" : "sdma";
        d["stream_gpu"] = r.stream_ordinal;
        d["bytes"] = r.bytes;
        d["reps"] = r.reps;
        d["ms"] = r.ms;
        d["gbps"] = r.gbps;
        d["verified"] = r.verified;
        return d;
      }, py::arg("src"), py::arg("dst"), py::arg("bytes"), py::arg("engine"), py::arg("reps") = 5,
      py::arg("stream_ordinal") = -1);
  m.def("measure_all_pairs", [](const std::vector<int>& ords, uint64_t bytes, int engine, int reps) {
        ConcurrentMeasure r;
        {
          py::gil_scoped_release rel;
          r = measure_all_pairs(ords, bytes, engine, reps);
        }
        py::dict d;
        d["gpus"] = r.gpus;
        d["copies"] = r.copies;
        d["engine"] = r.engine == kCopyKernel ? "kernel" : "sdma";
        d["bytes_per_copy"] = r.bytes_per_copy;
        d["wall_ms"] = r.wall_ms;
        d["aggregate_gbps"] = r.aggregate_gbps;
        d["per_copy_gbps"] = r.per_copy_gbps;
        d["verified"] = r.verified;
        return d;
      }, py::arg("ordinals"), py::arg("bytes"), py::arg("engine"), py::arg("reps") = 3);
  m.def("calibrate_copy_engines", &calibrate, py::arg("ordinals"), py::arg("sizes"), py::arg("reps") = 3,
        py::call_guard<py::gil_scoped_release>());
  m.def("choose_copy_engine", &choose_engine);
  m.def("set_copy_engine_override", &set_engine_override);
  m.def("copy_engine_table", &engine_table);
  m.def("record_copy_engine", &record_engine);

  py::class_<UserEvent>(m, "UserEvent")
      .def(py::init<>())
      .def("trigger", &UserEvent::trigger)
      .def_property_readonly("armed", &UserEvent::armed);

  py::class_<Cores, std::shared_ptr<Cores>>(m, "Cores")
      .def(py::init<const std::vector<DeviceInfo>&, const std::string&, const CoresConfig&>(),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("error_code", &Cores::error_code)
      .def_property_readonly("error_message", &Cores::error_message)
      .def_property_readonly("kernels", &Cores::kernels)
      .def_property_readonly("num_devices", &Cores::num_devices)
      .def_property_readonly("num_global_devices", &Cores::num_global_devices)
      .def_property_readonly("global_base", &Cores::global_base)
      .def_property_readonly("build_ms", &Cores::build_ms)
      .def("device", &Cores::device)
      .def("compute", &Cores::compute, py::call_guard<py::gil_scoped_release>())
      .def_property("enqueue_mode", &Cores::enqueue_mode,
                    [](Cores& c, bool on) {
                      py::gil_scoped_release r;
                      c.set_enqueue_mode(on);
                    })
      .def_readwrite("async_enqueue", &Cores::async_enqueue)
      .def_readwrite("no_compute", &Cores::no_compute)
      .def_readwrite("fine_grained", &Cores::fine_grained)
      .def_readwrite("smooth", &Cores::smooth)
      .def_readwrite("serial", &Cores::serial)
      .def_readwrite("peer_reads", &Cores::peer_reads)
      .def_readwrite("device_spans", &Cores::device_spans)
      .def_readwrite("deferred_downloads", &Cores::deferred_downloads)
      .def_readwrite("zc_release", &Cores::zc_release)
      .def_property("copy_cus", &Cores::copy_cus, &Cores::set_copy_cus)
      .def_readwrite("pipeline_writes_on_compute_stream", &Cores::pipeline_writes_on_compute_stream)
      .def_readwrite("pipeline_reads_on_main_stream", &Cores::pipeline_reads_on_main_stream)
      .def_readwrite("pipeline_reads_two_streams", &Cores::pipeline_reads_two_streams)
      .def_readwrite("sleep_waits", &Cores::sleep_waits)
      .def_readwrite("pipeline_writes_one_stream", &Cores::pipeline_writes_one_stream)
      .def_readwrite("driver_downloads_own_stream", &Cores::driver_downloads_own_stream)
      .def_readwrite("driver_reads_on_main_stream", &Cores::driver_reads_on_main_stream)
      .def_readwrite("inline_largest_share", &Cores::inline_largest_share)
      .def_readwrite("adaptive_sleep_waits", &Cores::adaptive_sleep_waits)
      .def_readwrite("sleep_wait_min_ms", &Cores::sleep_wait_min_ms)
      .def_readwrite("peer_read_min_bytes", &Cores::peer_read_min_bytes)
      .def_readwrite("graph_min_launches", &Cores::graph_min_launches)
      .def_readwrite("auto_failover", &Cores::auto_failover)
      .def_readwrite("record_schedule", &Cores::record_schedule)
      .def("schedule",
           [](Cores& c) {
             py::list out;
             for (auto& o : c.schedule())
               out.append(py::make_tuple(o.device, o.op, o.stream, o.begin, o.count, o.event));
             return out;
           })
      .def("clear_schedule", &Cores::clear_schedule)
      .def_property_readonly("failovers", &Cores::failovers)
      .def("set_device_enabled", &Cores::set_device_enabled)
      .def("device_enabled", &Cores::device_enabled)
      .def("inject_failure", &Cores::inject_failure)
      .def("gate", &Cores::gate, py::arg("event"), py::arg("device") = -1)
      .def_readwrite("dist_gather_writes", &Cores::dist_gather_writes)
      .def_readwrite("dist_broadcast_reads", &Cores::dist_broadcast_reads)
      .def_readwrite("dist_split_reads", &Cores::dist_split_reads)
      .def("set_time_scale", &Cores::set_time_scale)
      .def_readwrite("balancer_predictor", &Cores::balancer_predictor)
      .def("set_time_offset", &Cores::set_time_offset)
      .def("predictor_info", [](const Cores& c, int id) {
        py::dict d;
        const FitState* f = c.fit_state(id);
        if (!f) return d;
        d["decision"] = f->decision;
        d["a_ms"] = f->a;
        d["b_ms_per_item"] = f->b;
        d["o_multi_ms"] = f->o_multi;
        d["single_wall_ms"] = f->single_wall;
        d["predicted_multi_ms"] = f->predicted_multi_ms;
        d["measured_multi_ms"] = f->multi_wall;
        d["measured_law_ms"] = f->law_wall;
        return d;
      })
      .def("set_dynamic_lds", &Cores::set_dynamic_lds)
      .def("has_state", &Cores::has_state)
      .def("ranges", &Cores::ranges)
      .def("cpu_pool_id", &Cores::cpu_pool_id)
      .def("references", &Cores::references)
      .def("benchmarks", &Cores::benchmarks)
      .def("history", &Cores::history)
      .def("set_state", &Cores::set_state)
      .def("compute_ids", &Cores::compute_ids)
      .def_property_readonly("last_compute_id", &Cores::last_compute_id)
      .def("last_record", &Cores::last_record)
      .def_readwrite("record_timeline", &Cores::record_timeline)
      .def("set_device_enqueue_levels", &Cores::set_device_enqueue_levels)
      .def_property("debug_checks", &Cores::debug_checks, &Cores::set_debug_checks)
      .def("gemm_host_shells", &Cores::gemm_host_shells, py::call_guard<py::gil_scoped_release>())
      .def_property("kernel_d2h", &Cores::kernel_d2h, &Cores::set_kernel_d2h)
      .def_property("kernel_times_on", &Cores::kernel_times_on, &Cores::set_kernel_times)
      .def("kernel_times", &Cores::kernel_times, py::arg("device"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("kernel_d2h_bytes", &Cores::kernel_d2h_bytes)
      .def("device_enqueue_errors", &Cores::device_enqueue_errors, py::call_guard<py::gil_scoped_release>())
      .def("timeline",
           [](Cores& c) {
             std::vector<std::tuple<int, int, double, double, double, double>> out;
             std::vector<Cores::TimelineSpan> spans;
             {
               py::gil_scoped_release nogil;
               spans = c.timeline();
             }
             for (auto& s : spans)
               out.emplace_back(s.device, s.compute_id, s.begin_ms, s.end_ms, s.abs_begin_ms, s.abs_end_ms);
             return out;
           })
      .def("markers_reached", &Cores::markers_reached)
      .def("markers_issued", &Cores::markers_issued)
      .def("last_marker", &Cores::last_marker)
      .def("marker_word", &Cores::marker_word)
      .def("finish", &Cores::finish, py::call_guard<py::gil_scoped_release>())
      .def("capture_begin", &Cores::capture_begin, py::call_guard<py::gil_scoped_release>())
      .def("capture_end", &Cores::capture_end, py::call_guard<py::gil_scoped_release>())
      .def("graph_launch", &Cores::graph_launch, py::arg("id"), py::arg("times") = 1, py::arg("sync") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("graph_destroy", &Cores::graph_destroy, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("capturing", &Cores::capturing)
      .def("release_array", &Cores::release_array, py::call_guard<py::gil_scoped_release>())
      .def("device_bytes", &Cores::device_bytes)
      .def("device_pointer", &Cores::device_pointer)
      .def("upload", &Cores::upload, py::call_guard<py::gil_scoped_release>())
      .def("download", &Cores::download, py::call_guard<py::gil_scoped_release>())
      .def("copy_between", &Cores::copy_between, py::call_guard<py::gil_scoped_release>())
      .def("share_slices", &Cores::share_slices, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("peer_ordinals", &Cores::peer_ordinals)
      .def_property_readonly("peer_matrix", &Cores::peer_matrix)
      .def_property_readonly("p2p_path", &Cores::p2p_path)
      .def("can_peer", &Cores::can_peer)
      .def("set_distributed", &Cores::set_distributed);

  py::class_<PoolTask>(m, "PoolTask")
      .def(py::init<>())
      .def_property("call", &PoolTask::call, &PoolTask::set_call)
      .def_readwrite("type", &PoolTask::type)
      .def_readwrite("id", &PoolTask::id);

  py::class_<PoolCompletion>(m, "PoolCompletion")
      .def_readonly("id", &PoolCompletion::id)
      .def_readonly("device", &PoolCompletion::device)
      .def_readonly("ms", &PoolCompletion::ms)
      .def_readonly("error", &PoolCompletion::error);

  auto pool_cls = py::class_<DevicePool, std::shared_ptr<DevicePool>>(m, "DevicePool");
  pool_cls
      .def(py::init<std::vector<std::shared_ptr<Cores>>, int, int>(), py::arg("devices"), py::arg("max_in_flight"),
           py::arg("policy") = 0, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("policy", &DevicePool::policy)
      .def("enqueue", &DevicePool::enqueue, py::arg("tasks"), py::arg("pool_total") = -1, py::arg("append") = false,
           py::call_guard<py::gil_scoped_release>())
      // the batch form: task i = template calls[which[i]] with its own arrays,
      // type and id (one crossing and no per-task Python objects)
      .def("enqueue_batch",
           [](DevicePool& p, const std::vector<ComputeCall>& calls, const std::vector<int>& which,
              std::vector<std::vector<ArraySpec>> arrays, const std::vector<uint32_t>& types,
              const std::vector<long long>& ids, long long pool_total, bool append) {
             const size_t n = which.size();
             if (arrays.size() != n || types.size() != n || ids.size() != n)
               throw Error("enqueue_batch: which, arrays, types and ids must have one entry per task");
             std::vector<std::shared_ptr<const ComputeCall>> tmpl;
             tmpl.reserve(calls.size());
             for (const auto& c : calls) {
               auto t = std::make_shared<ComputeCall>(c);
               t->arrays.clear();
               tmpl.push_back(std::move(t));
             }
             std::vector<PoolTask> ts(n);
             for (size_t i = 0; i < n; ++i) {
               if (which[i] < 0 || static_cast<size_t>(which[i]) >= calls.size())
                 throw Error("enqueue_batch: template index out of range");
               ts[i].tmpl = tmpl[which[i]];
               ts[i].arrays = std::move(arrays[i]);
               ts[i].type = types[i];
               ts[i].id = ids[i];
             }
             py::gil_scoped_release r;
             p.enqueue(std::move(ts), pool_total, append);
           },
           py::arg("calls"), py::arg("which"), py::arg("arrays"), py::arg("types"), py::arg("ids"),
           py::arg("pool_total") = -1, py::arg("append") = false)
      .def("take_errors", &DevicePool::take_errors)
      .def("results",
           [](DevicePool& p, long long first, long long n) {
             std::vector<int> dev;
             std::vector<double> ms;
             p.results(first, n, dev, ms);
             return py::make_tuple(dev, ms);
           },
           py::arg("first"), py::arg("n"), "(devices, ms) of tasks [first, first + n); device -1: not retired")
      .attr("NOTIFY") = static_cast<uint32_t>(kTaskNotify);
  pool_cls
      .def("finish", &DevicePool::finish, py::call_guard<py::gil_scoped_release>())
      .def("completions", &DevicePool::completions, py::arg("timeout_ms") = 0.0,
           py::call_guard<py::gil_scoped_release>())
      .def("outstanding", &DevicePool::outstanding)
      .def("device_task_counts", &DevicePool::device_task_counts)
      .def("device_busy_ms", &DevicePool::device_busy_ms)
      .def("queue_limit", &DevicePool::queue_limit)
      .def("queue_limit_history", &DevicePool::queue_limit_history)
      .def("marker_speeds", &DevicePool::marker_speeds)
      .def("device_in_flight", &DevicePool::device_in_flight)
      .def("host_profile", &DevicePool::host_profile,
           "[issue ms, marker-poll ms, tasks issued, polls] summed over the consumer threads")
      .def_property_readonly("num_devices", &DevicePool::num_devices)
      .def_property_readonly("max_in_flight", &DevicePool::max_in_flight)
      .def("close", &DevicePool::close, py::call_guard<py::gil_scoped_release>());
}
