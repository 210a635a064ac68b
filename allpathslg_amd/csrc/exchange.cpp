// exchange.cpp — libapg's communicators: the byte exchange between the ranks
// of a sharded run (one process per GPU; k-mer-keyed shards; an
// all-to-all of records, all-gathers of solid sets / node sets, sums of
// spectra and counters).  ALLPATHS-LG itself has no collective layer
// (single-process OpenMP); this is the module boundary's
// multi-GPU form: apg_sharded_* (sharded.cpp) run every exchange here.
//
// Two transports behind one interface (apg.h "Communicators"):
//   rccl  device buffers over RCCL (xGMI inside a node): grouped
//         ncclSend / ncclRecv straight between the peer segments of the send
//         and receive buffers on the context's stream — every peer at once,
//         one xGMI link each — in pieces of at most kPiece bytes, so no single
//         transfer approaches 2^31 bytes; the segment to self is a device
//         copy (or, with APG_COMM_SELF_P2P, goes through RCCL too).  librccl
//         is opened at first use (the one torch may have loaded already is
//         reused by soname), so libapg needs it only for this transport.
//   tcp   host memory over TCP sockets (one full mesh, poll()-driven so every
//         peer's send and receive progress together).  With a context the
//         device segments are staged through pinned host buffers; without one
//         the buffers are host memory (the exchange's own CPU tests).  Used by
//         multi-process tests on one GPU and by the drop-in CLIs' bootstrap.
// Every size and offset is u64; byte counts per peer are explicit on both
// sides and checked against each other (a header per segment on tcp).
#include <arpa/inet.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "apg_core.hpp"
#include "exchange.hpp"

namespace apg {

// ---------------------------------------------------------------------------
// RCCL, resolved at run time
// ---------------------------------------------------------------------------
namespace {
typedef struct {
  char internal[128];
} NcclId;
typedef void* NcclComm;
enum { kNcclSuccess = 0, kNcclInProgress = 7 };
enum { kNcclUint8 = 1, kNcclUint32 = 3, kNcclUint64 = 5 };  // ncclDataType_t values (rccl.h)
enum { kNcclSum = 0, kNcclMax = 3 };       // ncclRedOp_t values

struct Nccl {
  bool ok = false;
  std::string err;
  int (*GetUniqueId)(NcclId*) = nullptr;
  int (*CommInitRank)(NcclComm*, int, NcclId, int) = nullptr;
  int (*CommDestroy)(NcclComm) = nullptr;
  int (*CommAbort)(NcclComm) = nullptr;
  int (*Send)(const void*, size_t, int, int, NcclComm, hipStream_t) = nullptr;
  int (*Recv)(void*, size_t, int, int, NcclComm, hipStream_t) = nullptr;
  int (*GroupStart)() = nullptr;
  int (*GroupEnd)() = nullptr;
  int (*AllReduce)(const void*, void*, size_t, int, int, NcclComm, hipStream_t) = nullptr;
  const char* (*GetErrorString)(int) = nullptr;
  int (*CommGetAsyncError)(NcclComm, int*) = nullptr;
};

Nccl& nccl() {
  static Nccl n = [] {
    Nccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      x.err = std::string("cannot open librccl: ") + dlerror();
      return x;
    }
#define APG_SYM(name, field)                                                      \
  x.field = reinterpret_cast<decltype(x.field)>(dlsym(h, name));                  \
  if (!x.field) {                                                                 \
    x.err = std::string("librccl lacks ") + name;                                 \
    return x;                                                                     \
  }
    APG_SYM("ncclGetUniqueId", GetUniqueId)
    APG_SYM("ncclCommInitRank", CommInitRank)
    APG_SYM("ncclCommDestroy", CommDestroy)
    APG_SYM("ncclCommAbort", CommAbort)
    APG_SYM("ncclSend", Send)
    APG_SYM("ncclRecv", Recv)
    APG_SYM("ncclGroupStart", GroupStart)
    APG_SYM("ncclGroupEnd", GroupEnd)
    APG_SYM("ncclAllReduce", AllReduce)
    APG_SYM("ncclGetErrorString", GetErrorString)
    APG_SYM("ncclCommGetAsyncError", CommGetAsyncError)
#undef APG_SYM
    x.ok = true;
    return x;
  }();
  return n;
}

#define APG_CHECK_NCCL(expr)                                                                       \
  do {                                                                                             \
    const int _r = (expr);                                                                         \
    if (_r != kNcclSuccess) {                                                                      \
      ::apg::set_error(std::string(#expr " failed: ") + nccl().GetErrorString(_r));                \
      return APG_E_HIP;                                                                            \
    }                                                                                              \
  } while (0)

}  // namespace

uint64_t Comm::piece_bytes() const { return kPiece; }

int Comm::alltoall_u64(const uint64_t* send, uint64_t* recv, uint64_t m) {
  if (world == 1) {  // a single rank: no staging through the device, no stream drain
    std::memmove(recv, send, m * 8);
    return APG_OK;
  }
  // small host arrays: m u64 per peer, through the host path of the transport
  std::vector<uint64_t> sb(world, m * 8), rb(world, m * 8);
  return alltoallv_host(send, sb.data(), recv, rb.data());
}

int Comm::allgather_u64(uint64_t v, std::vector<uint64_t>* all) {
  if (world == 1) {
    all->assign(1, v);
    return APG_OK;
  }
  all->assign(world, 0);
  std::vector<uint64_t> rb(world, 8);
  return allgatherv_host(&v, 8, all->data(), rb.data());
}

// ---------------------------------------------------------------------------
// RCCL transport
// ---------------------------------------------------------------------------
struct RcclComm : Comm {
  NcclComm nc = nullptr;
  bool self_p2p = false;
  unsigned long long* dsum = nullptr;  // small device staging (allreduce / host-path exchanges)
  uint64_t dsum_n = 0;

  int timeout_ms = 600000;

  ~RcclComm() override {
    if (nc) nccl().CommDestroy(nc);
    if (dsum) (void)hipFree(dsum);
  }

  void abort() override {
    if (nc) nccl().CommAbort(nc);
    nc = nullptr;
    aborted = true;
  }

  int live() {
    if (aborted) {
      set_error("apg_comm(rccl): the communicator was aborted");
      return APG_E_STATE;
    }
    return APG_OK;
  }

  // The collective's end: the stream drains, or RCCL reports a failed peer
  // (ncclCommGetAsyncError), or nothing finishes within timeout_ms — a rank
  // that died or aborted leaves its peers' kernels waiting forever, so a
  // plain hipStreamSynchronize would never return.  Failure aborts.
  int wait(const char* what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; ++spin) {
      const hipError_t q = hipStreamQuery(ctx->stream);
      if (q == hipSuccess) return APG_OK;
      if (q != hipErrorNotReady) {
        set_error(std::string("apg_comm(rccl): ") + what + ": " + hipGetErrorString(q));
        abort();
        return APG_E_HIP;
      }
      int e = kNcclSuccess;
      if (nccl().CommGetAsyncError(nc, &e) == kNcclSuccess && e != kNcclSuccess && e != kNcclInProgress) {
        set_error(std::string("apg_comm(rccl): ") + what + ": " + nccl().GetErrorString(e));
        abort();
        return APG_E_HIP;
      }
      if (std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
          timeout_ms) {
        set_error(std::string("apg_comm(rccl): ") + what + " timed out (a peer stopped)");
        abort();
        return APG_E_HIP;
      }
      if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }

  int stage(uint64_t n) {
    if (dsum_n >= n) return APG_OK;
    if (dsum) APG_CHECK_HIP(hipFree(dsum));
    dsum = nullptr;
    APG_CHECK_HIP(hipMalloc(&dsum, n * 8));
    dsum_n = n;
    return APG_OK;
  }

  // every peer's segments in one group: pieces of at most kPiece bytes.  A
  // failed Send / Recv still closes the group (an open group would swallow
  // the communicator's next calls).
  int p2p(const uint8_t* send, const uint64_t* sb, const uint64_t* soff, uint8_t* recv, const uint64_t* rb,
          const uint64_t* roff) {
    Nccl& N = nccl();
    APG_CHECK_NCCL(N.GroupStart());
    int r = kNcclSuccess;
    const char* what = "";
    for (int q = 0; q < world && r == kNcclSuccess; ++q) {
      if (q == rank && !self_p2p) continue;
      for (uint64_t o = 0; o < sb[q] && r == kNcclSuccess; o += kPiece) {
        r = N.Send(send + soff[q] + o, std::min<uint64_t>(kPiece, sb[q] - o), kNcclUint8, q, nc, ctx->stream);
        what = "ncclSend";
      }
      for (uint64_t o = 0; o < rb[q] && r == kNcclSuccess; o += kPiece) {
        r = N.Recv(recv + roff[q] + o, std::min<uint64_t>(kPiece, rb[q] - o), kNcclUint8, q, nc, ctx->stream);
        what = "ncclRecv";
      }
    }
    const int re = N.GroupEnd();
    if (r != kNcclSuccess) {
      set_error(std::string("apg_comm(rccl): ") + what + " failed: " + N.GetErrorString(r));
      return APG_E_HIP;
    }
    APG_CHECK_NCCL(re);
    return APG_OK;
  }

  // Unlike TCP (a length header per segment), point-to-point RCCL transfers
  // carry no sizes: a send / receive size mismatch between two ranks would
  // hang or overrun the receive segment.  Each rank's send sizes go to their
  // receivers first (a small host-path exchange) and are compared there.
  int check_sizes(const uint64_t* sb, const uint64_t* rb) {
    std::vector<uint64_t> peer_sb(world, 0);
    APG_TRY(alltoall_u64(sb, peer_sb.data(), 1));
    for (int q = 0; q < world; ++q)
      if (peer_sb[q] != rb[q]) {
        set_error("apg_comm(rccl): rank " + std::to_string(q) + " sends " + std::to_string(peer_sb[q]) + " bytes, " +
                  std::to_string(rb[q]) + " expected by rank " + std::to_string(rank));
        return APG_E_STATE;
      }
    return APG_OK;
  }

  int alltoallv(const void* send, const uint64_t* sb, void* recv, const uint64_t* rb) override {
    APG_TRY(live());
    APG_TRY(check_sizes(sb, rb));
    return alltoallv_raw(send, sb, recv, rb);
  }

  int alltoallv_raw(const void* send, const uint64_t* sb, void* recv, const uint64_t* rb) {
    std::vector<uint64_t> so(world + 1, 0), ro(world + 1, 0);
    for (int q = 0; q < world; ++q) {
      so[q + 1] = so[q] + sb[q];
      ro[q + 1] = ro[q] + rb[q];
    }
    APG_REQUIRE(sb[rank] == rb[rank], "apg_comm: the segment to self must have equal send and receive sizes");
    const auto* s = static_cast<const uint8_t*>(send);
    auto* r = static_cast<uint8_t*>(recv);
    if (!self_p2p && sb[rank])
      APG_CHECK_HIP(hipMemcpyAsync(r + ro[rank], s + so[rank], sb[rank], hipMemcpyDeviceToDevice, ctx->stream));
    APG_TRY(p2p(s, sb, so.data(), r, rb, ro.data()));
    return wait("alltoallv");
  }

  int allgatherv(const void* send, uint64_t bytes, void* recv, const uint64_t* rb) override {
    APG_TRY(live());
    std::vector<uint64_t> all;
    APG_TRY(allgather_u64(bytes, &all));
    for (int q = 0; q < world; ++q)
      if (all[q] != rb[q]) {
        set_error("apg_comm(rccl): rank " + std::to_string(q) + " gathers " + std::to_string(all[q]) + " bytes, " +
                  std::to_string(rb[q]) + " expected by rank " + std::to_string(rank));
        return APG_E_STATE;
      }
    return allgatherv_raw(send, bytes, recv, rb);
  }

  int allgatherv_raw(const void* send, uint64_t bytes, void* recv, const uint64_t* rb) {
    // every rank sends its segment to every peer: the all-to-all pattern of
    // xGMI's point-to-point links, exact sizes, no padding
    APG_REQUIRE(rb[rank] == bytes, "apg_comm_allgatherv: recv_bytes[rank] != send bytes");
    std::vector<uint64_t> sb(world, bytes), so(world, 0), ro(world + 1, 0);
    for (int q = 0; q < world; ++q) ro[q + 1] = ro[q] + rb[q];
    auto* r = static_cast<uint8_t*>(recv);
    if (!self_p2p && bytes)
      APG_CHECK_HIP(hipMemcpyAsync(r + ro[rank], send, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    APG_TRY(p2p(static_cast<const uint8_t*>(send), sb.data(), so.data(), r, rb, ro.data()));
    return wait("allgatherv");
  }

  int allreduce_u64(uint64_t* data, uint64_t n, int op) override {
    APG_TRY(live());
    if (!n || world == 1) return APG_OK;
    APG_TRY(stage(n));
    APG_CHECK_HIP(hipMemcpyAsync(dsum, data, n * 8, hipMemcpyHostToDevice, ctx->stream));
    APG_CHECK_NCCL(nccl().AllReduce(dsum, dsum, n, kNcclUint64, op == APG_COMM_MAX ? kNcclMax : kNcclSum, nc,
                                    ctx->stream));
    APG_TRY(wait("allreduce"));
    APG_CHECK_HIP(hipMemcpy(data, dsum, n * 8, hipMemcpyDeviceToHost));
    return APG_OK;
  }

  // in place on a device array (vote planes): ncclAllReduce in pieces
  int allreduce_dev_u32(uint32_t* d, uint64_t n) override {
    APG_TRY(live());
    const uint64_t piece = kPiece / 4;
    for (uint64_t o = 0; o < n; o += piece)
      APG_CHECK_NCCL(nccl().AllReduce(d + o, d + o, std::min<uint64_t>(piece, n - o), kNcclUint32, kNcclSum, nc,
                                      ctx->stream));
    return wait("allreduce");
  }

  // host-array exchanges (counts, sizes): staged through the device
  int alltoallv_host(const void* send, const uint64_t* sb, void* recv, const uint64_t* rb) override {
    APG_TRY(live());
    uint64_t ts = 0, tr = 0;
    for (int q = 0; q < world; ++q) ts += sb[q], tr += rb[q];
    APG_TRY(stage((ts + tr + 7) / 8 + 2));
    auto* d = reinterpret_cast<uint8_t*>(dsum);
    if (ts) APG_CHECK_HIP(hipMemcpyAsync(d, send, ts, hipMemcpyHostToDevice, ctx->stream));
    // host-path sizes are fixed by the caller's protocol (m u64 per peer)
    APG_TRY(alltoallv_raw(d, sb, d + ((ts + 7) & ~7ull), rb));
    if (tr) APG_CHECK_HIP(hipMemcpy(recv, d + ((ts + 7) & ~7ull), tr, hipMemcpyDeviceToHost));
    return APG_OK;
  }
  int allgatherv_host(const void* send, uint64_t bytes, void* recv, const uint64_t* rb) override {
    APG_TRY(live());
    uint64_t tr = 0;
    for (int q = 0; q < world; ++q) tr += rb[q];
    APG_TRY(stage((bytes + tr + 7) / 8 + 2));
    auto* d = reinterpret_cast<uint8_t*>(dsum);
    if (bytes) APG_CHECK_HIP(hipMemcpyAsync(d, send, bytes, hipMemcpyHostToDevice, ctx->stream));
    APG_TRY(allgatherv_raw(d, bytes, d + ((bytes + 7) & ~7ull), rb));
    if (tr) APG_CHECK_HIP(hipMemcpy(recv, d + ((bytes + 7) & ~7ull), tr, hipMemcpyDeviceToHost));
    return APG_OK;
  }
  int barrier() override {
    uint64_t x = 0;
    return allreduce_u64(&x, 1, APG_COMM_SUM);
  }
};

// ---------------------------------------------------------------------------
// TCP transport
// ---------------------------------------------------------------------------
namespace {

int set_nonblock(int fd, bool on) {
  const int fl = fcntl(fd, F_GETFL, 0);
  return fcntl(fd, F_SETFL, on ? (fl | O_NONBLOCK) : (fl & ~O_NONBLOCK));
}

bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

int tune(int fd) {
  int one = 1;
  (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  int buf = 8 << 20;
  (void)setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof buf);
  (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof buf);
  return fd;
}

int listen_on(const char* addr, int port, int* bound_port) {
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  int one = 1;
  (void)setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, addr, &sa.sin_addr) != 1) sa.sin_addr.s_addr = htonl(INADDR_ANY);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0 || ::listen(fd, 256) != 0) {
    ::close(fd);
    return -1;
  }
  socklen_t len = sizeof sa;
  ::getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &len);
  *bound_port = ntohs(sa.sin_port);
  return fd;
}

int connect_to(const char* host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host, std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      freeaddrinfo(res);
      return tune(fd);
    }
    if (fd >= 0) ::close(fd);
    if (std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
        timeout_ms) {
      freeaddrinfo(res);
      return -1;
    }
    usleep(20000);
  }
}

int accept_one(int lfd, int timeout_ms) {
  pollfd p{lfd, POLLIN, 0};
  const int k = ::poll(&p, 1, timeout_ms);
  if (k <= 0) return -1;
  const int fd = ::accept(lfd, nullptr, nullptr);
  return fd < 0 ? -1 : tune(fd);
}

}  // namespace

struct TcpComm : Comm {
  std::vector<int> fd;  // fd[q]: socket to peer q (-1 for self)
  int timeout_ms = 600000;
  uint8_t* hs = nullptr;  // pinned staging (device-memory communicators)
  uint8_t* hr = nullptr;
  uint64_t hs_n = 0, hr_n = 0;

  ~TcpComm() override {
    for (int f : fd)
      if (f >= 0) ::close(f);
    if (hs) (void)hipHostFree(hs);
    if (hr) (void)hipHostFree(hr);
  }

  // peers blocked in an exchange with this rank see the connection close
  void abort() override {
    for (int f : fd)
      if (f >= 0) ::shutdown(f, SHUT_RDWR);
    aborted = true;
  }

  int grow(uint8_t** p, uint64_t* have, uint64_t want) {
    if (*have >= want) return APG_OK;
    if (*p) APG_CHECK_HIP(hipHostFree(*p));
    *p = nullptr;
    *have = 0;
    const uint64_t n = std::max<uint64_t>(want + want / 8, 1 << 20);
    APG_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(p), n, 0));
    *have = n;
    return APG_OK;
  }

  // Every peer q at once: send out[q] (sb[q] bytes) and receive in[q] (rb[q]
  // bytes).  Each segment is preceded by its 8-byte length, checked on
  // arrival: a size mismatch between the two sides is an error, not a hang
  // or a silent truncation.
  int exchange(const std::vector<const uint8_t*>& out, const uint64_t* sb, const std::vector<uint8_t*>& in,
               const uint64_t* rb) {
    struct St {
      uint64_t hdr_out, hdr_in = 0;
      uint64_t sent = 0, got = 0;  // bytes incl. the 8-byte header
    };
    if (aborted) {
      set_error("apg_comm(tcp): the communicator was aborted");
      return APG_E_STATE;
    }
    std::vector<St> st(world);
    int pending = 0;
    for (int q = 0; q < world; ++q) {
      if (q == rank) continue;
      st[q].hdr_out = sb[q];
      set_nonblock(fd[q], true);
      ++pending;
    }
    auto t_last = std::chrono::steady_clock::now();
    int rc = APG_OK;
    while (pending > 0) {
      std::vector<pollfd> pf;
      std::vector<int> who;
      for (int q = 0; q < world; ++q) {
        if (q == rank) continue;
        const bool wsend = st[q].sent < 8 + sb[q], wrecv = st[q].got < 8 + rb[q];
        if (!wsend && !wrecv) continue;
        pf.push_back(pollfd{fd[q], (short)((wsend ? POLLOUT : 0) | (wrecv ? POLLIN : 0)), 0});
        who.push_back(q);
      }
      if (pf.empty()) break;
      const int k = ::poll(pf.data(), pf.size(), 1000);
      if (k < 0 && errno == EINTR) continue;
      if (k < 0) {
        set_error(std::string("apg_comm(tcp): poll failed: ") + strerror(errno));
        rc = APG_E_IO;
        break;
      }
      const auto now = std::chrono::steady_clock::now();
      if (k == 0) {
        if (std::chrono::duration_cast<std::chrono::milliseconds>(now - t_last).count() > timeout_ms) {
          set_error("apg_comm(tcp): exchange timed out (a peer stopped)");
          rc = APG_E_IO;
          break;
        }
        continue;
      }
      t_last = now;
      for (size_t i = 0; i < pf.size() && rc == APG_OK; ++i) {
        const int q = who[i];
        St& s = st[q];
        if (pf[i].revents & (POLLERR | POLLHUP | POLLNVAL) && !(pf[i].revents & POLLIN)) {
          set_error("apg_comm(tcp): peer " + std::to_string(q) + " closed the connection");
          rc = APG_E_IO;
          break;
        }
        if ((pf[i].revents & POLLOUT) && s.sent < 8 + sb[q]) {
          const uint8_t* src;
          size_t n;
          if (s.sent < 8) {
            src = reinterpret_cast<const uint8_t*>(&s.hdr_out) + s.sent;
            n = 8 - s.sent;
          } else {
            src = out[q] + (s.sent - 8);
            n = (size_t)std::min<uint64_t>(sb[q] - (s.sent - 8), 1 << 22);
          }
          const ssize_t w = ::send(fd[q], src, n, MSG_NOSIGNAL | MSG_DONTWAIT);
          if (w > 0) s.sent += (uint64_t)w;
          else if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
            set_error(std::string("apg_comm(tcp): send failed: ") + strerror(errno));
            rc = APG_E_IO;
          }
        }
        if ((pf[i].revents & POLLIN) && s.got < 8 + rb[q]) {
          uint8_t* dst;
          size_t n;
          if (s.got < 8) {
            dst = reinterpret_cast<uint8_t*>(&s.hdr_in) + s.got;
            n = 8 - s.got;
          } else {
            dst = in[q] + (s.got - 8);
            n = (size_t)std::min<uint64_t>(rb[q] - (s.got - 8), 1 << 22);
          }
          const ssize_t r = ::recv(fd[q], dst, n, MSG_DONTWAIT);
          if (r > 0) {
            s.got += (uint64_t)r;
            if (s.got == 8 && s.hdr_in != rb[q]) {
              set_error("apg_comm(tcp): peer " + std::to_string(q) + " sends " + std::to_string(s.hdr_in) +
                        " bytes, " + std::to_string(rb[q]) + " expected");
              rc = APG_E_STATE;
            }
          } else if (r == 0) {
            set_error("apg_comm(tcp): peer " + std::to_string(q) + " closed the connection");
            rc = APG_E_IO;
          } else if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) {
            set_error(std::string("apg_comm(tcp): recv failed: ") + strerror(errno));
            rc = APG_E_IO;
          }
        }
        if (s.sent == 8 + sb[q] && s.got == 8 + rb[q]) --pending;
      }
      if (rc != APG_OK) break;
    }
    for (int q = 0; q < world; ++q)
      if (q != rank) set_nonblock(fd[q], false);
    return rc;
  }

  int alltoallv_host(const void* send, const uint64_t* sb, void* recv, const uint64_t* rb) override {
    APG_REQUIRE(sb[rank] == rb[rank], "apg_comm: the segment to self must have equal send and receive sizes");
    std::vector<const uint8_t*> out(world);
    std::vector<uint8_t*> in(world);
    uint64_t so = 0, ro = 0;
    for (int q = 0; q < world; ++q) {
      out[q] = static_cast<const uint8_t*>(send) + so;
      in[q] = static_cast<uint8_t*>(recv) + ro;
      so += sb[q];
      ro += rb[q];
    }
    if (sb[rank]) std::memmove(in[rank], out[rank], sb[rank]);
    return exchange(out, sb, in, rb);
  }

  int allgatherv_host(const void* send, uint64_t bytes, void* recv, const uint64_t* rb) override {
    APG_REQUIRE(rb[rank] == bytes, "apg_comm_allgatherv: recv_bytes[rank] != send bytes");
    std::vector<const uint8_t*> out(world, static_cast<const uint8_t*>(send));
    std::vector<uint8_t*> in(world);
    std::vector<uint64_t> sb(world, bytes);
    uint64_t ro = 0;
    for (int q = 0; q < world; ++q) {
      in[q] = static_cast<uint8_t*>(recv) + ro;
      ro += rb[q];
    }
    if (bytes) std::memmove(in[rank], send, bytes);
    return exchange(out, sb.data(), in, rb);
  }

  int alltoallv(const void* send, const uint64_t* sb, void* recv, const uint64_t* rb) override {
    if (!ctx) return alltoallv_host(send, sb, recv, rb);
    uint64_t ts = 0, tr = 0;
    for (int q = 0; q < world; ++q) ts += sb[q], tr += rb[q];
    APG_TRY(grow(&hs, &hs_n, ts));
    APG_TRY(grow(&hr, &hr_n, tr));
    APG_CHECK_HIP(hipSetDevice(ctx->device));
    if (ts) APG_CHECK_HIP(hipMemcpyAsync(hs, send, ts, hipMemcpyDeviceToHost, ctx->stream));
    APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    APG_TRY(alltoallv_host(hs, sb, hr, rb));
    if (tr) APG_CHECK_HIP(hipMemcpyAsync(recv, hr, tr, hipMemcpyHostToDevice, ctx->stream));
    APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return APG_OK;
  }

  int allgatherv(const void* send, uint64_t bytes, void* recv, const uint64_t* rb) override {
    if (!ctx) return allgatherv_host(send, bytes, recv, rb);
    uint64_t tr = 0;
    for (int q = 0; q < world; ++q) tr += rb[q];
    APG_TRY(grow(&hs, &hs_n, bytes));
    APG_TRY(grow(&hr, &hr_n, tr));
    APG_CHECK_HIP(hipSetDevice(ctx->device));
    if (bytes) APG_CHECK_HIP(hipMemcpyAsync(hs, send, bytes, hipMemcpyDeviceToHost, ctx->stream));
    APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    APG_TRY(allgatherv_host(hs, bytes, hr, rb));
    if (tr) APG_CHECK_HIP(hipMemcpyAsync(recv, hr, tr, hipMemcpyHostToDevice, ctx->stream));
    APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return APG_OK;
  }

  int allreduce_u64(uint64_t* data, uint64_t n, int op) override {
    if (!n) return APG_OK;
    std::vector<uint64_t> all((size_t)n * world), rb(world, n * 8);
    APG_TRY(allgatherv_host(data, n * 8, all.data(), rb.data()));
    for (uint64_t i = 0; i < n; ++i) {
      uint64_t v = all[i];
      for (int q = 1; q < world; ++q) {
        const uint64_t x = all[(size_t)q * n + i];
        v = op == APG_COMM_MAX ? std::max(v, x) : v + x;
      }
      data[i] = v;
    }
    return APG_OK;
  }

  int barrier() override {
    uint64_t x = 0;
    return allreduce_u64(&x, 1, APG_COMM_SUM);
  }

  // Device array summed in place, in pieces of <= kDevPiece elements so the
  // pinned staging stays bounded (a 2^30-element consensus plane would pin
  // 8 GiB per rank): each piece staged through pinned memory, reduced as a
  // reduce-scatter (rank q sums slice q of every rank's piece) followed by an
  // all-gather of the summed slices, so no rank holds world copies.
  static constexpr uint64_t kDevPiece = 1ull << 25;  // 128 MiB of u32
  int allreduce_dev_u32(uint32_t* d, uint64_t n) override {
    for (uint64_t o = 0; o < n; o += kDevPiece) APG_TRY(allreduce_dev_piece(d + o, std::min(kDevPiece, n - o)));
    return APG_OK;
  }
  int allreduce_dev_piece(uint32_t* d, uint64_t n) {
    if (!n) return APG_OK;
    APG_REQUIRE(ctx, "apg_comm(tcp): device allreduce needs a context");
    std::vector<uint64_t> lo(world + 1);
    for (int q = 0; q <= world; ++q) lo[q] = n * (uint64_t)q / (uint64_t)world;
    const uint64_t mine = lo[rank + 1] - lo[rank];
    APG_TRY(grow(&hs, &hs_n, n * 4));
    APG_TRY(grow(&hr, &hr_n, std::max<uint64_t>(mine * 4 * world, n * 4)));
    APG_CHECK_HIP(hipSetDevice(ctx->device));
    APG_CHECK_HIP(hipMemcpyAsync(hs, d, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    std::vector<uint64_t> sb(world), rb(world, mine * 4);
    for (int q = 0; q < world; ++q) sb[q] = (lo[q + 1] - lo[q]) * 4;
    APG_TRY(alltoallv_host(hs, sb.data(), hr, rb.data()));
    auto* in = reinterpret_cast<const uint32_t*>(hr);
    std::vector<uint32_t> sum(in, in + mine);
    for (int q = 1; q < world; ++q)
      for (uint64_t i = 0; i < mine; ++i) sum[i] += in[(uint64_t)q * mine + i];
    std::vector<uint64_t> gb(world);
    for (int q = 0; q < world; ++q) gb[q] = (lo[q + 1] - lo[q]) * 4;
    APG_TRY(allgatherv_host(sum.data(), mine * 4, hs, gb.data()));
    APG_CHECK_HIP(hipMemcpyAsync(d, hs, n * 4, hipMemcpyHostToDevice, ctx->stream));
    APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
    return APG_OK;
  }

  // Full mesh: every rank listens on an ephemeral port and tells rank 0
  // (MASTER) its address; rank 0 sends the table back; rank i then connects to
  // every j < i and accepts every j > i, each connection opened by a
  // (rank, world) hello that is checked.
  int connect_mesh(const char* master, int port) {
    fd.assign(world, -1);
    if (world == 1) return APG_OK;
    int myport = 0;
    const int lfd = listen_on("0.0.0.0", 0, &myport);
    if (lfd < 0) {
      set_error(std::string("apg_comm(tcp): cannot listen: ") + strerror(errno));
      return APG_E_IO;
    }
    struct Ent {
      char host[64];
      int32_t port;
      int32_t rank;
    };
    std::vector<Ent> tab(world);
    int rc = APG_OK;
    char myhost[64] = {0};
    if (rank == 0) {
      int mport = 0;
      const int mfd = listen_on(master, port, &mport);
      if (mfd < 0) {
        ::close(lfd);
        set_error("apg_comm(tcp): rank 0 cannot listen on " + std::string(master) + ":" + std::to_string(port) +
                  ": " + strerror(errno));
        return APG_E_IO;
      }
      std::snprintf(tab[0].host, sizeof tab[0].host, "%s", master);
      tab[0].port = myport;
      tab[0].rank = 0;
      std::vector<int> tmp;
      for (int i = 1; i < world && rc == APG_OK; ++i) {
        const int f = accept_one(mfd, timeout_ms);
        Ent e{};
        if (f < 0 || !recv_all(f, &e, sizeof e) || e.rank <= 0 || e.rank >= world) {
          set_error("apg_comm(tcp): rank 0 did not hear from every rank");
          rc = APG_E_IO;
          if (f >= 0) ::close(f);
          break;
        }
        // the peer's address as rank 0 sees it
        sockaddr_in sa{};
        socklen_t len = sizeof sa;
        ::getpeername(f, reinterpret_cast<sockaddr*>(&sa), &len);
        inet_ntop(AF_INET, &sa.sin_addr, e.host, sizeof e.host);
        tab[e.rank] = e;
        tmp.push_back(f);
      }
      for (int f : tmp) {
        if (rc == APG_OK && !send_all(f, tab.data(), sizeof(Ent) * world)) rc = APG_E_IO;
        ::close(f);
      }
      ::close(mfd);
    } else {
      const int f = connect_to(master, port, timeout_ms);
      Ent e{};
      e.port = myport;
      e.rank = rank;
      if (f < 0 || !send_all(f, &e, sizeof e) || !recv_all(f, tab.data(), sizeof(Ent) * world)) {
        set_error("apg_comm(tcp): rank " + std::to_string(rank) + " cannot reach rank 0 at " + master + ":" +
                  std::to_string(port));
        rc = APG_E_IO;
      }
      if (f >= 0) ::close(f);
    }
    (void)myhost;
    for (int j = 0; j < rank && rc == APG_OK; ++j) {  // connect down
      const int f = connect_to(tab[j].host, tab[j].port, timeout_ms);
      int32_t hello[2] = {rank, world};
      if (f < 0 || !send_all(f, hello, sizeof hello)) {
        set_error("apg_comm(tcp): cannot connect to rank " + std::to_string(j));
        rc = APG_E_IO;
        if (f >= 0) ::close(f);
        break;
      }
      fd[j] = f;
    }
    for (int n = rank + 1; n < world && rc == APG_OK; ++n) {  // accept up
      const int f = accept_one(lfd, timeout_ms);
      int32_t hello[2];
      if (f < 0 || !recv_all(f, hello, sizeof hello) || hello[1] != world || hello[0] <= rank || hello[0] >= world ||
          fd[hello[0]] >= 0) {
        set_error("apg_comm(tcp): bad or missing connection from a higher rank");
        rc = APG_E_IO;
        if (f >= 0) ::close(f);
        break;
      }
      fd[hello[0]] = f;
    }
    ::close(lfd);
    return rc;
  }
};

}  // namespace apg

using namespace apg;

struct apg_comm {
  Comm* c;
};

extern "C" {

int apg_comm_unique_id(void* id128) {
  APG_REQUIRE(id128, "apg_comm_unique_id: NULL argument");
  Nccl& N = nccl();
  if (!N.ok) {
    set_error("apg_comm_unique_id: " + N.err);
    return APG_E_UNSUPPORTED;
  }
  NcclId id;
  APG_CHECK_NCCL(N.GetUniqueId(&id));
  std::memcpy(id128, &id, sizeof id);
  return APG_OK;
}

int apg_comm_init_rccl(apg_ctx* ctx, const void* id128, int rank, int world, uint32_t flags, apg_comm** out) {
  APG_REQUIRE(ctx && id128 && out, "apg_comm_init_rccl: NULL argument");
  APG_REQUIRE(world >= 1 && rank >= 0 && rank < world, "apg_comm_init_rccl: bad rank / world");
  *out = nullptr;
  Nccl& N = nccl();
  if (!N.ok) {
    set_error("apg_comm_init_rccl: " + N.err);
    return APG_E_UNSUPPORTED;
  }
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  auto* c = new (std::nothrow) RcclComm();
  if (!c) return APG_E_NOMEM;
  c->ctx = ctx;
  c->rank = rank;
  c->world = world;
  c->self_p2p = flags & APG_COMM_SELF_P2P;
  NcclId id;
  std::memcpy(&id, id128, sizeof id);
  const int r = N.CommInitRank(&c->nc, world, id, rank);
  if (r != kNcclSuccess) {
    set_error(std::string("ncclCommInitRank failed: ") + N.GetErrorString(r));
    c->nc = nullptr;
    delete c;
    return APG_E_HIP;
  }
  if (const char* e = std::getenv("APG_COMM_TIMEOUT_MS"))
    if (std::atoi(e) > 0) c->timeout_ms = std::atoi(e);
  *out = new (std::nothrow) apg_comm{c};
  if (!*out) {
    delete c;
    return APG_E_NOMEM;
  }
  return APG_OK;
}

int apg_comm_init_tcp(apg_ctx* ctx, const char* master_addr, int master_port, int rank, int world, int timeout_ms,
                      apg_comm** out) {
  APG_REQUIRE(master_addr && out, "apg_comm_init_tcp: NULL argument");
  APG_REQUIRE(world >= 1 && rank >= 0 && rank < world, "apg_comm_init_tcp: bad rank / world");
  APG_REQUIRE(master_port > 0 && master_port < 65536, "apg_comm_init_tcp: bad port");
  *out = nullptr;
  auto* c = new (std::nothrow) TcpComm();
  if (!c) return APG_E_NOMEM;
  c->ctx = ctx;
  c->rank = rank;
  c->world = world;
  if (timeout_ms > 0) c->timeout_ms = timeout_ms;
  const int rc = c->connect_mesh(master_addr, master_port);
  if (rc != APG_OK) {
    delete c;
    return rc;
  }
  *out = new (std::nothrow) apg_comm{c};
  if (!*out) {
    delete c;
    return APG_E_NOMEM;
  }
  return APG_OK;
}

int apg_comm_abort(apg_comm* comm) {
  APG_REQUIRE(comm, "apg_comm_abort: NULL argument");
  comm->c->abort();
  return APG_OK;
}

void apg_comm_destroy(apg_comm* comm) {
  if (!comm) return;
  delete comm->c;
  delete comm;
}

int apg_comm_rank(const apg_comm* comm) { return comm ? comm->c->rank : -1; }
int apg_comm_world(const apg_comm* comm) { return comm ? comm->c->world : -1; }

int apg_comm_alltoallv(apg_comm* comm, const void* send, const uint64_t* send_bytes, void* recv,
                       const uint64_t* recv_bytes) {
  APG_REQUIRE(comm && send_bytes && recv_bytes, "apg_comm_alltoallv: NULL argument");
  return comm->c->alltoallv(send, send_bytes, recv, recv_bytes);
}

int apg_comm_allgatherv(apg_comm* comm, const void* send, uint64_t send_bytes, void* recv,
                        const uint64_t* recv_bytes) {
  APG_REQUIRE(comm && recv_bytes, "apg_comm_allgatherv: NULL argument");
  return comm->c->allgatherv(send, send_bytes, recv, recv_bytes);
}

int apg_comm_allreduce_u64(apg_comm* comm, uint64_t* data, uint64_t n, int op) {
  APG_REQUIRE(comm && (data || !n), "apg_comm_allreduce_u64: NULL argument");
  APG_REQUIRE(op == APG_COMM_SUM || op == APG_COMM_MAX, "apg_comm_allreduce_u64: op must be SUM or MAX");
  return comm->c->allreduce_u64(data, n, op);
}

int apg_comm_barrier(apg_comm* comm) {
  APG_REQUIRE(comm, "apg_comm_barrier: NULL argument");
  return comm->c->barrier();
}

}  // extern "C"

namespace apg {
Comm* comm_of(apg_comm* c) { return c ? c->c : nullptr; }
}  // namespace apg
