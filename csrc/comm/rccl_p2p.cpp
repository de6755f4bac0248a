// Native RCCL point-to-point layer (pybind11 module `_comm`).
//
// The reference moves every activation over a fresh TCP connection through the
// dispatcher hub (`src/dispatcher.py:204-220`, `src/node.py:163-179`).  Here a
// stage pair exchanges device tensors with ncclSend/ncclRecv over xGMI on a
// communicator that has real failure semantics:
//
//  * non-blocking init: ncclCommInitRankConfig(blocking=0) returns at once and
//    is polled to completion, so a peer that never arrives can be abandoned;
//  * every enqueue (ncclGroupEnd on a non-blocking communicator) is polled with
//    the GIL released and an abort flag checked between polls;
//  * a watch thread polls ncclCommGetAsyncError and records (and optionally
//    acts on) the first asynchronous error;
//  * every ncclCommGetAsyncError of a communicator goes through one mutex: on a
//    non-blocking communicator that call also completes (joins) a finished
//    group job, and two threads (the watch thread and a waiter) joining the
//    same job at once is undefined -- the round-5 driver box hung in exactly
//    that pair of pollers;
//  * abort() = ncclCommAbort from any thread, after every other user of the
//    handle has left its poll loop (the handle is freed by the abort), run on a
//    helper thread with a deadline: an abort that does not return in time
//    (a kernel that never drains, a proxy thread stuck on a dead peer) leaves
//    the communicator marked `abort_stuck`, and the owner must give the
//    process up (report UNRECOVERABLE, exit non-zero) -- a fresh process, never
//    an exec, replaces it.
//
// The RCCL entry points are resolved with dlsym from the librccl that PyTorch
// already mapped (libtorch_hip needs it), so the process holds exactly one RCCL
// and our communicators live beside ProcessGroupNCCL's.
#include <dlfcn.h>
#include <link.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace py = pybind11;

namespace {

using Clock = std::chrono::steady_clock;

// Releases the GIL if this thread holds it.  The watch thread is a plain C++
// thread without a Python thread state: it may call abort(), and releasing a
// GIL it does not hold is undefined (a fatal error / crash in CPython).
struct NoGil {
  PyThreadState* st;
  NoGil() : st(PyGILState_Check() ? PyEval_SaveThread() : nullptr) {}
  NoGil(const NoGil&) = delete;
  NoGil& operator=(const NoGil&) = delete;
  ~NoGil() noexcept(false) {
    PyThreadState* s = st;
    st = nullptr;
    if (s) PyEval_RestoreThread(s);
  }
};

// ------------------------------------------------------------------ API table
struct Api {
  void* handle = nullptr;
  std::string path;
  decltype(&ncclGetVersion) getVersion = nullptr;
  decltype(&ncclGetUniqueId) getUniqueId = nullptr;
  decltype(&ncclCommInitRankConfig) initRankConfig = nullptr;
  decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommFinalize) finalize = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclBroadcast) bcast = nullptr;
  decltype(&ncclAllReduce) allReduce = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclGetLastError) lastError = nullptr;
};

Api g_api;
std::mutex g_api_mu;

int find_loaded(struct dl_phdr_info* info, size_t, void* data) {
  const char* name = info->dlpi_name;
  if (name && std::strstr(name, "librccl.so")) {
    *static_cast<std::string*>(data) = name;
    return 1;
  }
  return 0;
}

template <typename F>
void sym(F& slot, const char* name) {
  slot = reinterpret_cast<F>(dlsym(g_api.handle, name));
  if (!slot) throw std::runtime_error(std::string("rccl_p2p: librccl lacks ") + name);
}

// `hint` is the path PyTorch would load (torch/lib/librccl.so); an already
// mapped librccl always wins so the process never holds two copies.
const Api& api(const std::string& hint = "") {
  std::lock_guard<std::mutex> lk(g_api_mu);
  if (g_api.handle) return g_api;
  std::string path;
  dl_iterate_phdr(find_loaded, &path);
  void* h = nullptr;
  if (!path.empty()) h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
  if (!h && !hint.empty()) {
    h = dlopen(hint.c_str(), RTLD_NOW | RTLD_GLOBAL);
    path = hint;
  }
  if (!h) throw std::runtime_error("rccl_p2p: no librccl mapped in this process (import torch first)");
  g_api.handle = h;
  g_api.path = path;
  sym(g_api.getVersion, "ncclGetVersion");
  sym(g_api.getUniqueId, "ncclGetUniqueId");
  sym(g_api.initRankConfig, "ncclCommInitRankConfig");
  sym(g_api.getAsyncError, "ncclCommGetAsyncError");
  sym(g_api.abort, "ncclCommAbort");
  sym(g_api.finalize, "ncclCommFinalize");
  sym(g_api.destroy, "ncclCommDestroy");
  sym(g_api.send, "ncclSend");
  sym(g_api.recv, "ncclRecv");
  sym(g_api.bcast, "ncclBroadcast");
  sym(g_api.allReduce, "ncclAllReduce");
  sym(g_api.groupStart, "ncclGroupStart");
  sym(g_api.groupEnd, "ncclGroupEnd");
  sym(g_api.errorString, "ncclGetErrorString");
  sym(g_api.lastError, "ncclGetLastError");
  return g_api;
}

struct CommError : std::runtime_error {
  int code;
  CommError(const std::string& m, int c) : std::runtime_error(m), code(c) {}
};
struct CommAborted : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct CommTimeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ Comm
class Comm {
 public:
  Comm(const py::bytes& uid, int nranks, int rank, int device, bool blocking, const std::string& name)
      : nranks_(nranks), rank_(rank), device_(device), name_(name) {
    std::string u = uid;
    if (u.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("rccl_p2p: unique id must be 128 bytes");
    if (rank < 0 || rank >= nranks) throw std::invalid_argument("rccl_p2p: rank out of range");
    const Api& a = api();
    ncclUniqueId id;
    std::memcpy(&id, u.data(), sizeof(id));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = blocking ? 1 : 0;
    cfg.commName = name_.c_str();
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl_p2p: hipSetDevice failed");
    t_init_ = Clock::now();
    ncclResult_t r;
    {
      NoGil ng;
      r = a.initRankConfig(&comm_, nranks, id, rank, &cfg);
    }
    if (r != ncclSuccess && r != ncclInProgress) {
      // an init that failed synchronously may still have allocated the handle
      if (comm_) a.abort(comm_);
      comm_ = nullptr;
      throw CommError(std::string("ncclCommInitRankConfig: ") + a.errorString(r), (int)r);
    }
  }

  ~Comm() {
    stop_watch();
    // an unfinished object is abandoned, not finalized: finalize could wait on a dead peer
    if (comm_ && !aborted_.load()) abort();
    comm_ = nullptr;
  }

  // ncclResult_t of ncclCommGetAsyncError (7 = in progress), or -1 once aborted
  int poll() {
    Use u(this);
    if (!u.ok) return -1;
    ncclResult_t st = async_error();
    const int forced = forced_err_.load();
    if (forced != ncclSuccess && st == ncclSuccess) st = (ncclResult_t)forced;
    note(st);
    return (int)st;
  }

  // Fault injection for the failure-path tests: from now on the async-error
  // poll reports `code` as if RCCL had (a peer died mid-transfer, a remote
  // error): the watch thread sees it, records it and aborts the communicator.
  // On one GPU RCCL has no asynchronous error to provoke (the one local
  // misuse, a self-receive without its send, fails synchronously in
  // ncclGroupEnd).
  void inject_async_error(int code) { forced_err_.store(code); }

  // Block (GIL released) until every enqueued NCCL call is accepted; raise on
  // error, abort or timeout.  Covers init completion and ncclGroupEnd.
  void wait_ready(double timeout_s) {
    NoGil ng;
    wait_ready_nogil(timeout_s);
  }

  double init_ms() const { return init_ms_; }

  // Grouped p2p: ops = [(kind 's'|'r', device_ptr, nbytes, peer)], enqueued on `stream`.
  void p2p(const std::vector<std::tuple<std::string, uint64_t, uint64_t, int>>& ops, uint64_t stream,
           double timeout_s) {
    NoGil ng;
    Use u(this);
    if (!u.ok) throw CommAborted("rccl_p2p: communicator aborted");
    if (failed()) throw CommError("rccl_p2p: communicator failed: " + error_text(), err_.load());
    const Api& a = api();
    hipStream_t s = reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(stream));
    ncclResult_t r = a.groupStart();
    check(r, "ncclGroupStart");
    for (const auto& op : ops) {
      const std::string& kind = std::get<0>(op);
      void* ptr = reinterpret_cast<void*>(static_cast<uintptr_t>(std::get<1>(op)));
      size_t n = (size_t)std::get<2>(op);
      int peer = std::get<3>(op);
      if (peer < 0 || peer >= nranks_) {
        a.groupEnd();
        throw std::invalid_argument("rccl_p2p: peer out of range");
      }
      r = kind == "s" ? a.send(ptr, n, ncclUint8, peer, comm_, s) : a.recv(ptr, n, ncclUint8, peer, comm_, s);
      if (r != ncclSuccess && r != ncclInProgress) {
        a.groupEnd();
        check(r, kind == "s" ? "ncclSend" : "ncclRecv");
      }
      (kind == "s" ? bytes_sent_ : bytes_recv_) += n;
    }
    r = a.groupEnd();
    if (r != ncclSuccess && r != ncclInProgress) check(r, "ncclGroupEnd");
    ops_ += ops.size();
    wait_ready_inner(timeout_s);
  }

  // in-place broadcast of nbytes from `root` (weight push on (re)configuration)
  void broadcast(uint64_t ptr, uint64_t nbytes, int root, uint64_t stream, double timeout_s) {
    NoGil ng;
    Use u(this);
    if (!u.ok) throw CommAborted("rccl_p2p: communicator aborted");
    void* p = reinterpret_cast<void*>(static_cast<uintptr_t>(ptr));
    ncclResult_t r = api().bcast(p, p, (size_t)nbytes, ncclUint8, root, comm_,
                                 reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(stream)));
    if (r != ncclSuccess && r != ncclInProgress) check(r, "ncclBroadcast");
    wait_ready_inner(timeout_s);
  }

  // in-place fp32 max all-reduce (the bench's slowest-rank time)
  void allreduce_max_f32(uint64_t ptr, uint64_t count, uint64_t stream, double timeout_s) {
    NoGil ng;
    Use u(this);
    if (!u.ok) throw CommAborted("rccl_p2p: communicator aborted");
    void* p = reinterpret_cast<void*>(static_cast<uintptr_t>(ptr));
    ncclResult_t r = api().allReduce(p, p, (size_t)count, ncclFloat32, ncclMax, comm_,
                                     reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(stream)));
    if (r != ncclSuccess && r != ncclInProgress) check(r, "ncclAllReduce");
    wait_ready_inner(timeout_s);
  }

  // ncclCommAbort once every other user has left the handle; idempotent and
  // callable from any thread (the watch thread included).  Returns its latency.
  // The RCCL call runs on a detached helper thread and is waited for at most
  // `abort_deadline_s` (set_abort_deadline); past it the communicator is
  // marked abort_stuck and the handle is abandoned to the helper.
  double abort() {
    auto t0 = Clock::now();
    bool expected = false;
    if (!aborted_.compare_exchange_strong(expected, true)) return 0.0;
    {
      NoGil ng;
      // users poll the flag between polls (<= ~50 us); bounded in case one is stuck
      auto limit = Clock::now() + std::chrono::duration<double>(abort_deadline_s_.load());
      while (users_.load() > 0 && Clock::now() < limit) std::this_thread::sleep_for(std::chrono::microseconds(20));
      if (users_.load() > 0) abort_stuck_.store(true);     // a caller is stuck inside RCCL
      ncclComm_t c = comm_;
      comm_ = nullptr;
      if (c) {
        auto done = std::make_shared<std::atomic<int>>(0);
        const int stall_ms = abort_stall_ms_.load();
        std::thread([c, done, stall_ms] {
          if (stall_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(stall_ms));
          api().abort(c);
          done->store(1);
        }).detach();
        while (!done->load() && Clock::now() < limit) std::this_thread::sleep_for(std::chrono::microseconds(20));
        if (!done->load()) abort_stuck_.store(true);
      }
    }
    abort_ms_ = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    if (std::this_thread::get_id() != watch_id_) stop_watch();
    return abort_ms_;
  }

  // deadline of abort() (users leaving + ncclCommAbort), seconds
  void set_abort_deadline(double s) { abort_deadline_s_.store(s > 0.01 ? s : 0.01); }
  // Fault injection for the deadline path: the helper thread sleeps `ms`
  // before ncclCommAbort, standing in for an abort that RCCL never returns from.
  void inject_abort_stall(int ms) { abort_stall_ms_.store(ms); }

  // orderly teardown of a healthy communicator (all peers call it)
  void destroy(double timeout_s) {
    stop_watch();
    NoGil ng;
    bool expected = false;
    if (!aborted_.compare_exchange_strong(expected, true)) return;
    auto limit = Clock::now() + std::chrono::seconds(5);
    while (users_.load() > 0 && Clock::now() < limit) std::this_thread::sleep_for(std::chrono::microseconds(20));
    if (!comm_) return;
    const Api& a = api();
    ncclResult_t r = a.finalize(comm_);
    auto end = Clock::now() + std::chrono::duration<double>(timeout_s);
    ncclResult_t st = r;
    while (r == ncclSuccess || r == ncclInProgress) {
      st = async_error();
      if (st != ncclInProgress) break;
      if (Clock::now() > end) break;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (st == ncclSuccess) a.destroy(comm_);
    else a.abort(comm_);
    comm_ = nullptr;
  }

  // watch thread: poll ncclCommGetAsyncError every `period_us`; on the first
  // error record it and (abort_on_error) abort the communicator so every
  // pending wait returns
  void start_watch(int period_us, bool abort_on_error) {
    if (watching_.exchange(true)) return;
    watch_stop_ = false;
    int period = period_us < 50 ? 50 : period_us;
    watch_exited_ = false;
    watch_ = std::thread([this, period, abort_on_error] {
      watch_id_ = std::this_thread::get_id();
      while (!watch_stop_.load()) {
        int st = poll();
        if (st < 0) break;
        if (st != ncclSuccess && st != ncclInProgress) {
          if (abort_on_error) abort();
          break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(period));
      }
      watch_exited_ = true;
    });
  }

  // Joins the watch thread, bounded by the abort deadline: a watch thread
  // still inside an RCCL call past it is detached and the communicator is
  // marked abort_stuck (the process is to be given up).
  void stop_watch() {
    watch_stop_ = true;
    if (watch_.joinable() && std::this_thread::get_id() != watch_.get_id()) {
      NoGil ng;
      auto limit = Clock::now() + std::chrono::duration<double>(abort_deadline_s_.load());
      while (!watch_exited_.load() && Clock::now() < limit) std::this_thread::sleep_for(std::chrono::microseconds(50));
      if (watch_exited_.load()) {
        watch_.join();
      } else {
        abort_stuck_.store(true);
        watch_.detach();
      }
    }
    watching_ = false;
  }

  bool failed() const {
    int e = err_.load();
    return e != ncclSuccess && e != ncclInProgress;
  }
  bool aborted() const { return aborted_.load(); }
  bool abort_stuck() const { return abort_stuck_.load(); }
  double abort_ms() const { return abort_ms_; }
  int error_code() const { return err_.load(); }
  std::string error_text() {
    std::lock_guard<std::mutex> lk(msg_mu_);
    return err_msg_;
  }
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }
  int device() const { return device_; }
  uint64_t bytes_sent() const { return bytes_sent_.load(); }
  uint64_t bytes_recv() const { return bytes_recv_.load(); }
  uint64_t ops() const { return ops_.load(); }

 private:
  struct Use {
    Comm* c;
    bool ok;
    explicit Use(Comm* cm) : c(cm) {
      c->users_.fetch_add(1);
      ok = !c->aborted_.load() && c->comm_ != nullptr;
      if (!ok) c->users_.fetch_sub(1);
    }
    ~Use() {
      if (ok) c->users_.fetch_sub(1);
    }
  };

  // ncclCommGetAsyncError, serialized per communicator (see the file comment);
  // caller holds a Use (or is destroy(), after every user left)
  ncclResult_t async_error() {
    std::lock_guard<std::mutex> lk(poll_mu_);
    ncclResult_t st = ncclSuccess;
    ncclResult_t r = api().getAsyncError(comm_, &st);
    return r != ncclSuccess ? r : st;
  }

  void note(ncclResult_t st) {
    if (st == ncclSuccess || st == ncclInProgress) return;
    int expected = ncclSuccess;
    if (err_.compare_exchange_strong(expected, (int)st)) {
      std::lock_guard<std::mutex> lk(msg_mu_);
      const char* last = comm_ ? api().lastError(comm_) : nullptr;
      err_msg_ = std::string(api().errorString(st)) + (last && *last ? std::string(": ") + last : "");
    }
  }

  void check(ncclResult_t r, const char* what) {
    if (r == ncclSuccess || r == ncclInProgress) return;
    note(r);
    throw CommError(std::string(what) + ": " + error_text(), (int)r);
  }

  void wait_ready_nogil(double timeout_s) {
    Use u(this);
    if (!u.ok) throw CommAborted("rccl_p2p: communicator aborted");
    wait_ready_inner(timeout_s);
  }

  // caller holds a Use
  void wait_ready_inner(double timeout_s) {
    auto end = Clock::now() + std::chrono::duration<double>(timeout_s);
    int spins = 0;
    while (true) {
      if (aborted_.load()) throw CommAborted("rccl_p2p: communicator aborted");
      ncclResult_t st = async_error();
      if (st == ncclSuccess && forced_err_.load() != ncclSuccess) st = (ncclResult_t)forced_err_.load();
      if (st == ncclSuccess) break;
      if (st != ncclInProgress) {
        note(st);
        throw CommError("rccl_p2p: " + error_text(), (int)st);
      }
      if (Clock::now() > end) throw CommTimeout("rccl_p2p: operation still in progress after timeout");
      if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (!ready_) {
      ready_ = true;
      init_ms_ = std::chrono::duration<double, std::milli>(Clock::now() - t_init_).count();
    }
  }

  ncclComm_t comm_ = nullptr;
  int nranks_, rank_, device_;
  std::string name_;
  std::atomic<bool> aborted_{false};
  std::atomic<bool> abort_stuck_{false};
  std::atomic<double> abort_deadline_s_{3.0};
  std::atomic<int> abort_stall_ms_{0};
  double abort_ms_ = 0.0;
  std::mutex poll_mu_;
  std::atomic<int> users_{0};
  std::atomic<int> err_{ncclSuccess};
  std::atomic<int> forced_err_{ncclSuccess};
  std::mutex msg_mu_;
  std::string err_msg_;
  std::thread watch_;
  std::thread::id watch_id_;
  std::atomic<bool> watch_stop_{false};
  std::atomic<bool> watch_exited_{true};
  std::atomic<bool> watching_{false};
  std::atomic<uint64_t> bytes_sent_{0}, bytes_recv_{0}, ops_{0};
  Clock::time_point t_init_;
  bool ready_ = false;
  double init_ms_ = -1.0;
};

}  // namespace

PYBIND11_MODULE(_comm, m) {
  m.doc() = "ADAPT native RCCL point-to-point layer: non-blocking communicators, grouped send/recv, "
            "async-error watch, abort";
  // leaked on purpose: these type objects must outlive interpreter teardown
  static auto* exc_err = new py::exception<CommError>(m, "CommError", PyExc_RuntimeError);
  static auto* exc_ab = new py::exception<CommAborted>(m, "CommAborted", PyExc_RuntimeError);
  static auto* exc_to = new py::exception<CommTimeout>(m, "CommTimeout", PyExc_TimeoutError);
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const CommError& e) {
      // instance carries the ncclResult_t as `.code`
      PyObject* inst = PyObject_CallFunction(exc_err->ptr(), "s", e.what());
      if (inst) {
        PyObject* code = PyLong_FromLong(e.code);
        PyObject_SetAttrString(inst, "code", code);
        Py_XDECREF(code);
        PyErr_SetObject(exc_err->ptr(), inst);
        Py_DECREF(inst);
      }
    } catch (const CommAborted& e) {
      (*exc_ab)(e.what());
    } catch (const CommTimeout& e) {
      (*exc_to)(e.what());
    }
  });

  m.def("load", [](const std::string& hint) { return api(hint).path; }, py::arg("hint") = "",
        "resolve the RCCL entry points (from the librccl PyTorch mapped); returns its path");
  m.def("version", []() {
    int v = 0;
    api().getVersion(&v);
    return v;
  });
  m.def("unique_id", []() {
    ncclUniqueId id;
    ncclResult_t r;
    {
      NoGil ng;
      r = api().getUniqueId(&id);
    }
    if (r != ncclSuccess) throw CommError(std::string("ncclGetUniqueId: ") + api().errorString(r), (int)r);
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  m.attr("IN_PROGRESS") = (int)ncclInProgress;
  m.attr("SUCCESS") = (int)ncclSuccess;

  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def(py::init<const py::bytes&, int, int, int, bool, const std::string&>(), py::arg("uid"),
           py::arg("nranks"), py::arg("rank"), py::arg("device"), py::arg("blocking") = false,
           py::arg("name") = "adapt")
      .def("poll", &Comm::poll)
      .def("wait_ready", &Comm::wait_ready, py::arg("timeout_s") = 30.0)
      .def("p2p", &Comm::p2p, py::arg("ops"), py::arg("stream"), py::arg("timeout_s") = 30.0)
      .def("broadcast", &Comm::broadcast, py::arg("ptr"), py::arg("nbytes"), py::arg("root"), py::arg("stream"),
           py::arg("timeout_s") = 30.0)
      .def("allreduce_max_f32", &Comm::allreduce_max_f32, py::arg("ptr"), py::arg("count"), py::arg("stream"),
           py::arg("timeout_s") = 30.0)
      .def("abort", &Comm::abort)
      .def("destroy", &Comm::destroy, py::arg("timeout_s") = 10.0)
      .def("start_watch", &Comm::start_watch, py::arg("period_us") = 1000, py::arg("abort_on_error") = true)
      .def("inject_async_error", &Comm::inject_async_error, py::arg("code") = (int)ncclRemoteError)
      .def("stop_watch", &Comm::stop_watch)
      .def("set_abort_deadline", &Comm::set_abort_deadline, py::arg("seconds"))
      .def("inject_abort_stall", &Comm::inject_abort_stall, py::arg("ms"))
      .def_property_readonly("abort_stuck", &Comm::abort_stuck)
      .def_property_readonly("abort_ms", &Comm::abort_ms)
      .def_property_readonly("failed", &Comm::failed)
      .def_property_readonly("aborted", &Comm::aborted)
      .def_property_readonly("error_code", &Comm::error_code)
      .def_property_readonly("error_text", &Comm::error_text)
      .def_property_readonly("init_ms", &Comm::init_ms)
      .def_property_readonly("nranks", &Comm::nranks)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("device", &Comm::device)
      .def_property_readonly("bytes_sent", &Comm::bytes_sent)
      .def_property_readonly("bytes_recv", &Comm::bytes_recv)
      .def_property_readonly("ops", &Comm::ops);
}
