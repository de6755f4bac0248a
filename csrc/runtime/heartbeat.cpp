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
#include <utility>
#include <vector>

#include "runtime.h"

namespace adapt_rt {

namespace {
using Clock = std::chrono::steady_clock;

struct Sender {
  int fd = -1;
  std::atomic<bool> stop{false};
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
      ++seq;
      (void)send(s->fd, msg.data(), msg.size(), MSG_DONTWAIT);   // a lost datagram is just a missed beat
      std::this_thread::sleep_for(std::chrono::microseconds(period));
    }
  });
  return s;
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
      std::string id(buf, strnlen(buf, static_cast<size_t>(n)));
      std::lock_guard<std::mutex> g(m->mu);
      m->last[id] = Clock::now();
      m->count[id] += 1;
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

void hb_monitor_forget(void* h, const std::string& id) {
  auto* m = static_cast<Monitor*>(h);
  std::lock_guard<std::mutex> g(m->mu);
  m->last.erase(id);
  m->count.erase(id);
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
