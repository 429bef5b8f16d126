// net.h — blocking TCP helpers shared by the bootstrap (bootstrap.cc) and the
// negotiation channel (negotiate.cc). Host-side control messages only: no tensor
// bytes ever travel here (they go over RCCL / xGMI).
#pragma once

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <stdlib.h>

#include <atomic>
#include <string>

namespace tips {
namespace net {

inline bool send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n > 0) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

inline bool recv_all(int fd, void* buf, size_t n, int timeout_ms) {
  char* p = static_cast<char*>(buf);
  while (n > 0) {
    pollfd pfd{fd, POLLIN, 0};
    int pr = ::poll(&pfd, 1, timeout_ms);
    if (pr < 0 && errno == EINTR) continue;
    if (pr <= 0) return false;
    ssize_t k = ::recv(fd, p, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

inline bool resolve(const char* host, int port, sockaddr_in* out) {
  memset(out, 0, sizeof *out);
  out->sin_family = AF_INET;
  out->sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host, &out->sin_addr) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host, nullptr, &hints, &res) != 0 || !res) return false;
  out->sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}


// Listening socket on all interfaces; -1 and *err on failure.
inline int listen_on(int port, int backlog, std::string* err) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) {
    *err = std::string("socket: ") + strerror(errno);
    return -1;
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  sa.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0 || ::listen(fd, backlog) != 0) {
    *err = "bind/listen on port " + std::to_string(port) + ": " + strerror(errno);
    ::close(fd);
    return -1;
  }
  return fd;
}

// Length-prefixed message (u32 little-endian length + bytes).
inline bool send_msg(int fd, const std::string& m) {
  uint32_t n = (uint32_t)m.size();
  return send_all(fd, &n, sizeof n) && send_all(fd, m.data(), m.size());
}

inline bool recv_msg(int fd, std::string* m, int timeout_ms) {
  uint32_t n = 0;
  if (!recv_all(fd, &n, sizeof n, timeout_ms) || n > (64u << 20)) return false;
  m->resize(n);
  return n == 0 || recv_all(fd, &(*m)[0], n, timeout_ms);
}

// A connect() to a loopback port in the ephemeral range with no listener can succeed by TCP
// simultaneous open with ITSELF (source port == destination port). A retry loop that connects
// before the listener is up is exposed to it: the "connection" then carries our own hello back
// to us and the listener never hears from this rank. Such a socket must be closed and retried.
inline bool connected_to_self(int fd) {
  sockaddr_in a{}, b{};
  socklen_t la = sizeof a, lb = sizeof b;
  if (getsockname(fd, reinterpret_cast<sockaddr*>(&a), &la) != 0 ||
      getpeername(fd, reinterpret_cast<sockaddr*>(&b), &lb) != 0)
    return false;
  return a.sin_port == b.sin_port && a.sin_addr.s_addr == b.sin_addr.s_addr;
}

inline void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

// Join counters (tips_net_stats): connections a joining rank dropped because they reached itself,
// and connections rank 0 dropped because the joiner never confirmed them.
inline std::atomic<int64_t>& self_connects() {
  static std::atomic<int64_t> n{0};
  return n;
}
inline std::atomic<int64_t>& unconfirmed_joins() {
  static std::atomic<int64_t> n{0};
  return n;
}

// A joining rank's connect to sa, for both joins (bootstrap, negotiation). Returns a connected
// socket that did not reach itself, or -1. TIPS_TEST_SELF_CONNECT=n (tests only): the first n
// attempts of the process bind their source port to the destination port first, so that with no
// listener there yet the connect completes as a TCP simultaneous open with itself - the case the
// check below exists for, made deterministic.
inline int connect_peer(const sockaddr_in& sa) {
  static std::atomic<int> forced{-1};
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  if (forced.load() < 0) {
    const char* v = getenv("TIPS_TEST_SELF_CONNECT");
    int expect = -1;
    forced.compare_exchange_strong(expect, v ? atoi(v) : 0);
  }
  if (forced.load() > 0) {
    forced--;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in me = sa;
    me.sin_addr.s_addr = sa.sin_addr.s_addr;
    (void)::bind(fd, reinterpret_cast<const sockaddr*>(&me), sizeof me);  // (fails once a listener holds the port)
  }
  if (::connect(fd, reinterpret_cast<const sockaddr*>(&sa), sizeof sa) != 0) {
    ::close(fd);
    return -1;
  }
  if (connected_to_self(fd)) {
    self_connects()++;
    ::close(fd);
    return -1;
  }
  return fd;
}

}  // namespace net
}  // namespace tips
