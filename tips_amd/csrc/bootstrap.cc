// bootstrap.cc — hands the RCCL unique id from rank 0 to every rank over TCP.
//
// Replaces what the reference needs MPI_Init + an MPI-broadcast IP table +
// ZeroMQ port exchange for (tips/core/mpi/tips_mpi.cc:14-29,
// tips/core/common/naive_rpc.cc:201-246): on one node with one process per
// GPU the only thing ranks must agree on before RCCL exists is the 128-byte
// ncclUniqueId. Rank 0 listens, every other rank connects (retrying until a
// deadline), says who it is, and receives the id.
#include "net.h"

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

namespace tips {

using namespace net;

constexpr uint8_t kIdAck = 0xA5;  // a joining rank's confirmation that it has the id


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
      uint8_t ack = 0;
      if (!recv_all(c, &peer, sizeof peer, std::min(ms_left(), 5000)) || peer <= 0 || peer >= size ||
          !send_all(c, id, (size_t)id_bytes)) {
        ::close(c);
        continue;
      }
      // a rank counts as joined only once it confirms it has the id: a send can succeed into the
      // socket of a rank that has already given up on this attempt (it then asks again, and this
      // loop must still be listening for it)
      if (!recv_all(c, &ack, 1, std::min(ms_left(), 5000)) || ack != kIdAck) {
        unconfirmed_joins()++;
        ::close(c);
        continue;
      }
      if (!seen[peer]) {  // a rank that asks again just gets the id again
        seen[peer] = true;
        joined++;
      }
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
  static std::atomic<int> drop_first{-1};  // TIPS_TEST_DROP_FIRST_HELLO=1 (tests only): give up on the first
  if (drop_first.load() < 0) {             // connection right after asking, as a rank whose answer timed out
    const char* v = getenv("TIPS_TEST_DROP_FIRST_HELLO");
    int expect = -1;
    drop_first.compare_exchange_strong(expect, v ? atoi(v) : 0);
  }
  while (true) {
    const int fd = connect_peer(sa);  // (-1: refused, or it reached itself)
    if (fd >= 0) {
      const int32_t me = rank;
      const uint8_t ack = kIdAck;
      if (send_all(fd, &me, sizeof me) && drop_first.load() > 0) {
        drop_first--;
        ::close(fd);
        continue;
      }
      // a bounded wait: a listener that never answers (another program's socket on this port) costs
      // one attempt, not the whole timeout
      const bool ok = recv_all(fd, id, (size_t)id_bytes, std::min(ms_left(), 5000)) && send_all(fd, &ack, 1);
      ::close(fd);
      if (ok) return 0;
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
