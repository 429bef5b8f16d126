// bootstrap.cc — hands the RCCL unique id from rank 0 to every rank over TCP.
//
// Replaces what the reference needs MPI_Init + an MPI-broadcast IP table +
// ZeroMQ port exchange for (tips/core/mpi/tips_mpi.cc:14-29,
// tips/core/common/naive_rpc.cc:201-246): on one node with one process per
// GPU the only thing ranks must agree on before RCCL exists is the 128-byte
// ncclUniqueId. Rank 0 listens, every other rank connects (retrying until a
// deadline), says who it is, and receives the id.
#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

namespace tips {

namespace {

bool send_all(int fd, const void* buf, size_t n) {
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

bool recv_all(int fd, void* buf, size_t n, int timeout_ms) {
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

bool resolve(const char* host, int port, sockaddr_in* out) {
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

}  // namespace

// Returns 0 on success; on failure fills *err and returns -1.
int bootstrap_exchange(int rank, int size, const char* host, int port, void* id, int id_bytes, int timeout_s,
                       std::string* err) {
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  auto ms_left = [&]() {
    auto d = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now()).count();
    return d > 0 ? (int)d : 0;
  };
  if (size <= 1) return 0;
  if (rank == 0) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
      *err = std::string("bootstrap: socket: ") + strerror(errno);
      return -1;
    }
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
    if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0 || ::listen(fd, size) != 0) {
      *err = "bootstrap: bind/listen on port " + std::to_string(port) + ": " + strerror(errno);
      ::close(fd);
      return -1;
    }
    std::vector<bool> seen(size, false);
    int joined = 0;
    while (joined < size - 1) {
      pollfd pfd{fd, POLLIN, 0};
      int pr = ::poll(&pfd, 1, ms_left());
      if (pr < 0 && errno == EINTR) continue;
      if (pr <= 0) {
        *err = "bootstrap: timed out waiting for " + std::to_string(size - 1 - joined) + " rank(s)";
        ::close(fd);
        return -1;
      }
      int c = ::accept(fd, nullptr, nullptr);
      if (c < 0) continue;
      int32_t peer = -1;
      if (!recv_all(c, &peer, sizeof peer, ms_left()) || peer <= 0 || peer >= size || seen[peer] ||
          !send_all(c, id, (size_t)id_bytes)) {
        ::close(c);
        continue;
      }
      seen[peer] = true;
      joined++;
      ::close(c);
    }
    ::close(fd);
    return 0;
  }
  sockaddr_in sa;
  if (!resolve(host, port, &sa)) {
    *err = std::string("bootstrap: cannot resolve ") + host;
    return -1;
  }
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
      *err = std::string("bootstrap: socket: ") + strerror(errno);
      return -1;
    }
    if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) == 0) {
      int32_t me = rank;
      bool ok = send_all(fd, &me, sizeof me) && recv_all(fd, id, (size_t)id_bytes, ms_left());
      ::close(fd);
      if (ok) return 0;
    } else {
      ::close(fd);
    }
    if (ms_left() == 0) {
      *err = "bootstrap: rank " + std::to_string(rank) + " could not reach rank 0 at " + host + ":" +
             std::to_string(port);
      return -1;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

}  // namespace tips
