// pybind11 module `_runtime`: framing transport + LZ4 frame + reversible zfp.
// Every call releases the GIL around its native work so the dispatcher's and
// workers' I/O threads run concurrently (the reference's threads serialize on
// the GIL inside pure-Python chunk loops, `src/node_state.py:70-89`).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>

#include "runtime.h"

namespace py = pybind11;
using namespace adapt_rt;

// GIL release whose destructor may propagate the forced unwind that CPython
// 3.10 uses to retire a daemon thread returning from native code during
// interpreter finalization (pybind11's gil_scoped_release destructor is
// noexcept, which turns that unwind into std::terminate).
struct NoGil {
  PyThreadState* st;
  NoGil() : st(PyEval_SaveThread()) {}
  NoGil(const NoGil&) = delete;
  NoGil& operator=(const NoGil&) = delete;
  ~NoGil() noexcept(false) {
    PyThreadState* s = st;
    st = nullptr;
    if (s) PyEval_RestoreThread(s);
  }
};

static py::bytes to_bytes(const std::vector<uint8_t>& v) {
  return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
}

static std::pair<const uint8_t*, size_t> view(const py::buffer& b, py::buffer_info& info) {
  info = b.request();
  return {static_cast<const uint8_t*>(info.ptr), (size_t)(info.size * info.itemsize)};
}

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "ADAPT host runtime: framing transport, LZ4 frame codec, reversible zfp-style codec";

  // ---------------------------------------------------------- bulk copy
  // dst[:n] = src[:n] on `threads` threads, GIL released: the dispatcher copies every
  // request into a shared-memory ingest slot (19 MB per bs=32 fp32 batch), which one
  // thread's memcpy makes the serving bottleneck
  m.def("copy_into", [](py::buffer dst, py::buffer src, int threads) {
    py::buffer_info di = dst.request(true), si = src.request();
    const size_t n = (size_t)(si.size * si.itemsize);
    if ((size_t)(di.size * di.itemsize) < n) throw std::runtime_error("copy_into: destination too small");
    uint8_t* d = static_cast<uint8_t*>(di.ptr);
    const uint8_t* sp = static_cast<const uint8_t*>(si.ptr);
    NoGil ng;
    parallel_copy(d, sp, n, threads);
  });

  // ---------------------------------------------------------- heartbeats
  m.def("hb_sender_start", [](const std::string& host, int port, const std::string& id, int period_us) {
    return reinterpret_cast<uintptr_t>(hb_sender_start(host, port, id, period_us));
  });
  m.def("hb_sender_stop", [](uintptr_t h) {
    NoGil nogil;
    hb_sender_stop(reinterpret_cast<void*>(h));
  });
  m.def("hb_sender_progress", [](uintptr_t h, uint64_t v, uint64_t stage_ns, uint64_t epoch) {
    hb_sender_progress(reinterpret_cast<void*>(h), v, stage_ns, epoch);
  }, py::arg("h"), py::arg("value"), py::arg("stage_ns") = 0, py::arg("epoch") = 0);
  m.def("hb_monitor_progress", [](uintptr_t h) { return hb_monitor_progress(reinterpret_cast<void*>(h)); });
  m.def("hb_monitor_start", [](int port) { return reinterpret_cast<uintptr_t>(hb_monitor_start(port)); });
  m.def("hb_monitor_port", [](uintptr_t h) { return hb_monitor_port(reinterpret_cast<void*>(h)); });
  m.def("hb_monitor_ages", [](uintptr_t h) { return hb_monitor_ages(reinterpret_cast<void*>(h)); });
  m.def("hb_monitor_forget", [](uintptr_t h, const std::string& id) {
    hb_monitor_forget(reinterpret_cast<void*>(h), id);
  });
  m.def("hb_monitor_stop", [](uintptr_t h) {
    NoGil nogil;
    hb_monitor_stop(reinterpret_cast<void*>(h));
  });

  // ------------------------------------------------------------- framing
  m.def("send_frame", [](int fd, py::buffer data, size_t chunk, int timeout_ms) {
    py::buffer_info info;
    auto v = view(data, info);
    NoGil nogil;
    send_frame(fd, v.first, v.second, chunk, timeout_ms);
  }, py::arg("fd"), py::arg("data"), py::arg("chunk") = 512000, py::arg("timeout_ms") = -1);
  m.def("send_frame_parts", [](int fd, py::list parts, size_t chunk, int timeout_ms) {
    std::vector<py::buffer_info> infos;
    std::vector<std::pair<const uint8_t*, size_t>> v;
    infos.reserve(parts.size());
    for (auto h : parts) {
      py::buffer b = py::reinterpret_borrow<py::buffer>(h);
      infos.emplace_back();
      auto pv = view(b, infos.back());
      v.emplace_back(pv.first, pv.second);
    }
    NoGil nogil;
    send_frame_parts(fd, v, chunk, timeout_ms);
  }, py::arg("fd"), py::arg("parts"), py::arg("chunk") = 512000, py::arg("timeout_ms") = -1);
  m.def("send_all", [](int fd, py::buffer data, size_t chunk, int timeout_ms) {
    py::buffer_info info;
    auto v = view(data, info);
    NoGil nogil;
    send_all(fd, v.first, v.second, chunk, timeout_ms);
  }, py::arg("fd"), py::arg("data"), py::arg("chunk") = 512000, py::arg("timeout_ms") = -1);
  m.def("recv_frame", [](int fd, size_t chunk, int timeout_ms, size_t max_len) -> py::object {
    // header first, then receive straight into an uninitialised bytes object:
    // no zero-fill, no staging vector, no second copy (a 57 MB frame used to
    // pay two fresh-page faults passes, a memset and a memcpy)
    uint8_t hdr[8];
    uint64_t n = 0;
    bool ok;
    {
      NoGil nogil;
      ok = recv_exact(fd, hdr, 8, 8, timeout_ms, true);
    }
    if (!ok) return py::none();
    for (int i = 0; i < 8; ++i) n = (n << 8) | hdr[i];
    if (max_len && n > max_len) throw std::runtime_error("frame larger than max_len");
    PyObject* b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)n);
    if (!b) throw py::error_already_set();
    py::object obj = py::reinterpret_steal<py::object>(b);
    if (n) {
      uint8_t* dst = reinterpret_cast<uint8_t*>(PyBytes_AS_STRING(b));
      NoGil nogil;
      recv_exact(fd, dst, (size_t)n, chunk, timeout_ms, false);
    }
    return obj;
  }, py::arg("fd"), py::arg("chunk") = 512000, py::arg("timeout_ms") = -1, py::arg("max_len") = 0);
  m.def("recv_exact", [](int fd, size_t n, int timeout_ms) -> py::object {
    std::vector<uint8_t> out(n);
    bool ok;
    {
      NoGil nogil;
      ok = recv_exact(fd, out.data(), n, n ? n : 1, timeout_ms, true);
    }
    if (!ok) return py::none();
    return to_bytes(out);
  }, py::arg("fd"), py::arg("n"), py::arg("timeout_ms") = -1);
  m.def("recv_frame_into", [](int fd, py::buffer dst, size_t chunk, int timeout_ms) -> py::object {
    // receive a frame directly into a writable buffer (e.g. pinned host memory)
    py::buffer_info info = dst.request(true);
    size_t cap = (size_t)(info.size * info.itemsize);
    uint8_t hdr[8];
    uint64_t n = 0;
    bool ok;
    {
      NoGil nogil;
      ok = recv_exact(fd, hdr, 8, 8, timeout_ms, true);
      if (ok) {
        for (int i = 0; i < 8; ++i) n = (n << 8) | hdr[i];
        if (n > cap) throw std::runtime_error("frame larger than destination buffer");
        if (n) recv_exact(fd, static_cast<uint8_t*>(info.ptr), (size_t)n, chunk, timeout_ms, false);
      }
    }
    if (!ok) return py::none();
    return py::int_(n);
  }, py::arg("fd"), py::arg("dst"), py::arg("chunk") = 512000, py::arg("timeout_ms") = -1);

  // ---------------------------------------------------------------- LZ4
  m.def("xxh32", [](py::buffer data, uint32_t seed) {
    py::buffer_info info;
    auto v = view(data, info);
    return xxh32(v.first, v.second, seed);
  }, py::arg("data"), py::arg("seed") = 0);
  m.def("lz4_compress", [](py::buffer data, int accel) {
    py::buffer_info info;
    auto v = view(data, info);
    std::vector<uint8_t> out;
    {
      NoGil nogil;
      out = lz4_frame_compress(v.first, v.second, accel);
    }
    return to_bytes(out);
  }, py::arg("data"), py::arg("accel") = 1);
  m.def("lz4_decompress", [](py::buffer data) {
    py::buffer_info info;
    auto v = view(data, info);
    std::vector<uint8_t> out;
    {
      NoGil nogil;
      out = lz4_frame_decompress(v.first, v.second);
    }
    return to_bytes(out);
  });
  m.def("lz4_frame_blocks", [](py::buffer data) {
    py::buffer_info info;
    auto v = view(data, info);
    Lz4FrameBlocks b = lz4_frame_blocks(v.first, v.second);
    py::array_t<uint32_t> offs(b.offsets.size()), words(b.words.size());
    if (!b.offsets.empty()) {
      std::memcpy(offs.mutable_data(), b.offsets.data(), b.offsets.size() * 4);
      std::memcpy(words.mutable_data(), b.words.data(), b.words.size() * 4);
    }
    return py::make_tuple(b.content_size, b.block_max, b.independent, offs, words);
  });
  m.def("lz4_block_compress", [](py::buffer data, int accel) {
    py::buffer_info info;
    auto v = view(data, info);
    std::vector<uint8_t> out(lz4_block_bound(v.second));
    size_t n;
    {
      NoGil nogil;
      n = lz4_block_compress(v.first, v.second, out.data(), out.size(), accel);
    }
    out.resize(n);
    return to_bytes(out);
  }, py::arg("data"), py::arg("accel") = 1);
  m.def("lz4_block_decompress", [](py::buffer data, size_t max_out) {
    py::buffer_info info;
    auto v = view(data, info);
    std::vector<uint8_t> out(max_out);
    size_t n;
    {
      NoGil nogil;
      n = lz4_block_decompress(v.first, v.second, out.data(), out.size());
    }
    out.resize(n);
    return to_bytes(out);
  });

  // ---------------------------------------------------------------- zvc
  m.def("zvc_compress", [](py::buffer data, int esz) {
    py::buffer_info info;
    auto v = view(data, info);
    if (v.second % esz) throw std::runtime_error("zvc_compress: byte length not a multiple of the element size");
    std::vector<uint8_t> out;
    {
      NoGil nogil;
      out = zvc_compress(v.first, v.second / esz, esz);
    }
    return to_bytes(out);
  }, py::arg("data"), py::arg("esz") = 2);
  m.def("zvc_info", [](py::buffer data) {
    py::buffer_info info;
    auto v = view(data, info);
    ZvcHeader h = zvc_header(v.first, v.second);
    py::array_t<uint32_t> offs(h.offsets.size());
    if (!h.offsets.empty()) std::memcpy(offs.mutable_data(), h.offsets.data(), h.offsets.size() * 4);
    return py::make_tuple(h.n, h.esz, h.nseg, offs);
  });
  m.def("zvc_decompress", [](py::buffer data) {
    py::buffer_info info;
    auto v = view(data, info);
    ZvcHeader h = zvc_header(v.first, v.second);
    std::vector<uint8_t> out(h.n * h.esz);
    {
      NoGil nogil;
      zvc_decompress(v.first, v.second, out.data());
    }
    return to_bytes(out);
  });

  // ---------------------------------------------------------------- zfp
  m.def("zfp_compress", [](py::array arr, int threads, size_t chunk_blocks) {
    py::buffer_info info = arr.request();
    int code;
    if (info.format == py::format_descriptor<float>::format() && info.itemsize == 4) code = 0;
    else if (info.format == py::format_descriptor<double>::format() && info.itemsize == 8) code = 1;
    else throw std::runtime_error("zfp_compress: float32 or float64 arrays only");
    if (!(arr.flags() & py::array::c_style)) throw std::runtime_error("zfp_compress: array must be C-contiguous");
    std::vector<size_t> shape;
    for (auto s : info.shape) shape.push_back((size_t)s);
    if (shape.empty()) shape.push_back(1);
    std::vector<uint8_t> out;
    {
      NoGil nogil;
      out = zfp_compress(info.ptr, code, shape, threads, chunk_blocks);
    }
    return to_bytes(out);
  }, py::arg("arr"), py::arg("threads") = 4, py::arg("chunk_blocks") = 0);
  m.def("zfp_info", [](py::buffer data) {
    py::buffer_info info;
    auto v = view(data, info);
    ZfpHeader h = zfp_header(v.first, v.second);
    return py::make_tuple(h.dtype, h.shape, h.payload_off, h.chunk_blocks);
  });
  m.def("zfp_decompress", [](py::buffer data, int threads) {
    py::buffer_info info;
    auto v = view(data, info);
    ZfpHeader h = zfp_header(v.first, v.second);
    std::vector<ssize_t> shape(h.shape.begin(), h.shape.end());
    py::array out = h.dtype == 0 ? py::array(py::dtype::of<float>(), shape) : py::array(py::dtype::of<double>(), shape);
    void* dst = out.mutable_data();
    {
      NoGil nogil;
      zfp_decompress(v.first, v.second, dst, threads);
    }
    return out;
  }, py::arg("data"), py::arg("threads") = 4);
}
