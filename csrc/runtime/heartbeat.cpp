// Native liveness heartbeats (UDP), free of the Python GIL.
//
// A SIGKILLed worker's sockets are closed by the kernel only after its address
// space (GPU mappings included) has been torn down, which on a busy MI355X
// takes 100+ ms; its membership lease expires only after the TTL.  A sender
// thread in the worker emits a datagram every `period_us`; the dispatcher's
// monitor thread timestamps arrivals per worker id, and the dispatcher polls
// the ages: a worker silent for a few periods has stopped executing.  Both
// threads are plain C++ threads, so a worker busy in Python (GIL held by the
// compute loop) keeps beating.
//
// Every datagram also carries the worker's completed-micro-batch counter
// (`hb_sender_progress`).  A worker whose heartbeat thread runs but whose
// counter stands still while its pipeline holds work is *hung* (a wedged GPU
// queue, a deadlocked compute loop): the monitor timestamps each counter change
// so the dispatcher can tell a stalled stage from a dead one (the reference's
// per-hop `start_time` registry serves that purpose, `src/dispatcher.py:186-194`).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

#include "runtime.h"

namespace adapt_rt {

namespace {
using Clock = std::chrono::steady_clock;

struct Sender {
  int fd = -1;
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> progress{0};
  std::atomic<uint64_t> stage_ns{0};                    // the worker's measured time per micro-batch
  std::atomic<uint64_t> epoch{0};                       // epoch the counter belongs to
  std::thread th;
};

struct Monitor {
  int fd = -1;
  int port = 0;
  std::atomic<bool> stop{false};
  std::thread th;
  std::mutex mu;
  std::map<std::string, Clock::time_point> last;
  std::map<std::string, uint64_t> count;
  std::map<std::string, uint64_t> prog;                 // last reported progress counter
  std::map<std::string, Clock::time_point> prog_t;      // when it last changed
  std::map<std::string, uint64_t> stage_ns;             // reported time per micro-batch (0 = unknown)
  std::map<std::string, uint64_t> epoch;                // epoch of the reported counter
};
}  // namespace

void* hb_sender_start(const std::string& host, int port, const std::string& id, int period_us) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_DGRAM;
  if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || res == nullptr)
    throw std::runtime_error("hb_sender_start: cannot resolve " + host);
  int fd = socket(AF_INET, SOCK_DGRAM, 0);
  if (fd < 0 || connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
    freeaddrinfo(res);
    if (fd >= 0) close(fd);
    throw std::runtime_error("hb_sender_start: cannot open the heartbeat socket");
  }
  freeaddrinfo(res);
  auto* s = new Sender();
  s->fd = fd;
  const int period = period_us < 500 ? 500 : period_us;
  s->th = std::thread([s, id, period] {
    uint64_t seq = 0;
    std::string msg;
    while (!s->stop.load(std::memory_order_relaxed)) {
      msg = id;
      msg.push_back('\0');
      msg.append(reinterpret_cast<const char*>(&seq), sizeof(seq));
      const uint64_t prog = s->progress.load(std::memory_order_relaxed);
      msg.append(reinterpret_cast<const char*>(&prog), sizeof(prog));
      const uint64_t sns = s->stage_ns.load(std::memory_order_relaxed);
      msg.append(reinterpret_cast<const char*>(&sns), sizeof(sns));
      const uint64_t ep = s->epoch.load(std::memory_order_relaxed);
      msg.append(reinterpret_cast<const char*>(&ep), sizeof(ep));
      ++seq;
      (void)send(s->fd, msg.data(), msg.size(), MSG_DONTWAIT);   // a lost datagram is just a missed beat
      std::this_thread::sleep_for(std::chrono::microseconds(period));
    }
  });
  return s;
}

void hb_sender_progress(void* h, uint64_t value, uint64_t stage_ns, uint64_t epoch) {
  auto* s = static_cast<Sender*>(h);
  if (s == nullptr) return;
  s->epoch.store(epoch, std::memory_order_relaxed);
  s->progress.store(value, std::memory_order_relaxed);
  if (stage_ns) s->stage_ns.store(stage_ns, std::memory_order_relaxed);
}

void hb_sender_stop(void* h) {
  auto* s = static_cast<Sender*>(h);
  if (s == nullptr) return;
  s->stop.store(true);
  if (s->th.joinable()) s->th.join();
  close(s->fd);
  delete s;
}

void* hb_monitor_start(int port) {
  int fd = socket(AF_INET, SOCK_DGRAM, 0);
  if (fd < 0) throw std::runtime_error("hb_monitor_start: socket failed");
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
    close(fd);
    throw std::runtime_error("hb_monitor_start: bind failed");
  }
  socklen_t len = sizeof(a);
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
  auto* m = new Monitor();
  m->fd = fd;
  m->port = ntohs(a.sin_port);
  m->th = std::thread([m] {
    char buf[512];
    while (!m->stop.load(std::memory_order_relaxed)) {
      pollfd p{m->fd, POLLIN, 0};
      if (poll(&p, 1, 20) <= 0) continue;
      ssize_t n = recv(m->fd, buf, sizeof(buf) - 1, MSG_DONTWAIT);
      if (n <= 0) continue;
      buf[n] = 0;
      const size_t idlen = strnlen(buf, static_cast<size_t>(n));
      std::string id(buf, idlen);
      const auto now = Clock::now();
      std::lock_guard<std::mutex> g(m->mu);
      m->last[id] = now;
      m->count[id] += 1;
      if (static_cast<size_t>(n) >= idlen + 1 + 2 * sizeof(uint64_t)) {
        uint64_t prog = 0, ep = 0;
        std::memcpy(&prog, buf + idlen + 1 + sizeof(uint64_t), sizeof(prog));
        if (static_cast<size_t>(n) >= idlen + 1 + 4 * sizeof(uint64_t))
          std::memcpy(&ep, buf + idlen + 1 + 3 * sizeof(uint64_t), sizeof(ep));
        auto it = m->prog.find(id);
        if (it == m->prog.end() || it->second != prog || m->epoch[id] != ep) {
          m->prog[id] = prog;
          m->prog_t[id] = now;
          m->epoch[id] = ep;
        }
        if (static_cast<size_t>(n) >= idlen + 1 + 3 * sizeof(uint64_t)) {
          uint64_t sns = 0;
          std::memcpy(&sns, buf + idlen + 1 + 2 * sizeof(uint64_t), sizeof(sns));
          m->stage_ns[id] = sns;
        }
      }
    }
  });
  return m;
}

int hb_monitor_port(void* h) { return static_cast<Monitor*>(h)->port; }

std::vector<std::pair<std::string, double>> hb_monitor_ages(void* h) {
  auto* m = static_cast<Monitor*>(h);
  std::vector<std::pair<std::string, double>> out;
  const auto now = Clock::now();
  std::lock_guard<std::mutex> g(m->mu);
  for (const auto& kv : m->last)
    out.emplace_back(kv.first, std::chrono::duration<double>(now - kv.second).count());
  return out;
}

std::vector<std::tuple<std::string, uint64_t, double, double, uint64_t>> hb_monitor_progress(void* h) {
  auto* m = static_cast<Monitor*>(h);
  std::vector<std::tuple<std::string, uint64_t, double, double, uint64_t>> out;
  const auto now = Clock::now();
  std::lock_guard<std::mutex> g(m->mu);
  for (const auto& kv : m->prog)
    out.emplace_back(kv.first, kv.second, std::chrono::duration<double>(now - m->prog_t[kv.first]).count(),
                     static_cast<double>(m->stage_ns[kv.first]) * 1e-9, m->epoch[kv.first]);
  return out;
}

void hb_monitor_forget(void* h, const std::string& id) {
  auto* m = static_cast<Monitor*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  m->last.erase(id);
  m->count.erase(id);
  m->prog.erase(id);
  m->prog_t.erase(id);
  m->stage_ns.erase(id);
  m->epoch.erase(id);
}

void hb_monitor_stop(void* h) {
  auto* m = static_cast<Monitor*>(h);
  if (m == nullptr) return;
  m->stop.store(true);
  if (m->th.joinable()) m->th.join();
  close(m->fd);
  delete m;
}

}  // namespace adapt_rt
