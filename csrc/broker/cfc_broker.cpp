// cfc-broker: a single-node topic-exchange message broker (C++17, epoll, one event-loop thread).
//
// What it replaces: the reference's RabbitMQ (infra/rabbitmq/definitions.json: one topic exchange
// `copilot.events`, one durable queue per routing key; publisher confirms + persistent messages,
// rabbitmq_publisher.py:148-156,370-378; manual ack / nack(requeue), rabbitmq_subscriber.py:
// 504-560).  The services of this framework speak to it through bus/cfcbroker.py when they run as
// separate processes (one per service, as the reference's compose topology does) on a node that
// has no RabbitMQ.  Semantics kept:
//   * topic exchanges with `*` (one word) and `#` (zero or more words) binding patterns;
//   * durable queues: every enqueue / settle is journaled (append-only file per queue, group-commit
//     fdatasync once per event-loop turn) BEFORE the publisher's confirm is sent, and replayed on
//     restart -- a confirmed message survives a broker crash;
//   * per-consumer prefetch (basic.qos), round-robin over a queue's consumers, ack / nack(requeue);
//     a consumer's connection dropping requeues its unacked messages at the head of the queue;
//   * a redelivery limit (the reference only counts a DLQ metric, event_handler.py:120-175): a
//     message nacked / orphaned more than `max_redeliveries` times, or nacked without requeue, moves
//     to `<queue>.dlq` -- what tools/failed_queues.py inspects, requeues and purges.
//
// Wire protocol (all integers big-endian):  frame = u32 len | u8 op | payload (len = 1 + payload).
//   str = u16 len + bytes, blob = u32 len + bytes.  Every request carries a u32 request id that the
//   reply echoes; DELIVER frames are unsolicited.  See bus/cfcbroker.py for the client side.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cctype>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace {

enum Op : uint8_t {
  OP_HELLO = 1, OP_OK = 2, OP_ERR = 3,
  OP_DECLARE = 10, OP_BIND = 11, OP_UNBIND = 12, OP_DELETE = 13, OP_PURGE = 14,
  OP_PUBLISH = 20, OP_CONFIRM = 21,
  OP_CONSUME = 30, OP_CANCEL = 31, OP_DELIVER = 32, OP_ACK = 33, OP_NACK = 34,
  OP_GET = 40, OP_GET_OK = 41, OP_PEEK = 42, OP_PEEK_OK = 43,
  OP_STATS = 50, OP_STATS_OK = 51,
  OP_PING = 60, OP_PONG = 61,
};

constexpr uint32_t kMaxFrame = 64u << 20;          // 64 MiB
constexpr size_t kWriteHighWater = 8u << 20;       // stop delivering to a connection above this
constexpr uint32_t kProtocolVersion = 1;

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- wire encoding
struct Writer {
  std::string b;
  void u8(uint8_t v) { b.push_back((char)v); }
  void u16(uint16_t v) { u8(v >> 8); u8(v & 0xff); }
  void u32(uint32_t v) { u16(v >> 16); u16(v & 0xffff); }
  void u64(uint64_t v) { u32((uint32_t)(v >> 32)); u32((uint32_t)v); }
  void str(const std::string& s) { u16((uint16_t)s.size()); b.append(s); }
  void blob(const std::string& s) { u32((uint32_t)s.size()); b.append(s); }
};

struct Reader {
  const char* p;
  size_t n, off = 0;
  bool ok = true;
  Reader(const char* p_, size_t n_) : p(p_), n(n_) {}
  bool need(size_t k) {
    if (!ok || off + k > n) { ok = false; return false; }
    return true;
  }
  uint8_t u8() { if (!need(1)) return 0; return (uint8_t)p[off++]; }
  uint16_t u16() { uint16_t a = u8(); return (uint16_t)((a << 8) | u8()); }
  uint32_t u32() { uint32_t a = u16(); return (a << 16) | u16(); }
  uint64_t u64() { uint64_t a = u32(); return (a << 32) | u32(); }
  std::string str() { size_t k = u16(); if (!need(k)) return {}; std::string s(p + off, k); off += k; return s; }
  std::string blob() { size_t k = u32(); if (!need(k)) return {}; std::string s(p + off, k); off += k; return s; }
};

std::string frame(uint8_t op, const std::string& payload) {
  Writer w;
  w.u32((uint32_t)(1 + payload.size()));
  w.u8(op);
  w.b.append(payload);
  return std::move(w.b);
}

bool valid_name(const std::string& s) {
  if (s.empty() || s.size() > 255) return false;
  for (unsigned char c : s)
    if (c < 0x21 || c == 0x7f || c == '/') return false;
  return true;
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o.push_back('\\'); o.push_back((char)c); }
    else if (c < 0x20) { char t[8]; snprintf(t, sizeof t, "\\u%04x", c); o.append(t); }
    else o.push_back((char)c);
  }
  return o;
}

std::vector<std::string> split_words(const std::string& s) {
  std::vector<std::string> out;
  size_t a = 0;
  for (;;) {
    size_t b = s.find('.', a);
    out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) break;
    a = b + 1;
  }
  return out;
}

// AMQP topic match: `*` = exactly one word, `#` = zero or more words
bool topic_match(const std::vector<std::string>& p, size_t i, const std::vector<std::string>& k, size_t j) {
  while (i < p.size()) {
    if (p[i] == "#") {
      if (i + 1 == p.size()) return true;
      for (size_t jj = j; jj <= k.size(); ++jj)
        if (topic_match(p, i + 1, k, jj)) return true;
      return false;
    }
    if (j >= k.size()) return false;
    if (p[i] != "*" && p[i] != k[j]) return false;
    ++i;
    ++j;
  }
  return j == k.size();
}

// ---------------------------------------------------------------- broker state
struct Msg {
  uint64_t id = 0;
  uint32_t redeliv = 0;
  std::string rk;
  std::shared_ptr<const std::string> body;
};

struct Conn;

struct Consumer {
  Conn* conn;
  std::string queue;
  uint32_t prefetch;   // 0 = unlimited
  uint32_t inflight = 0;
};

struct Binding {
  std::string exchange, pattern;
  std::vector<std::string> words;
};

struct Queue {
  std::string name;
  bool durable = true;
  uint32_t max_redeliv = 5;
  std::deque<Msg> ready;
  std::unordered_map<uint64_t, Msg> inflight;   // delivered, not yet settled
  std::vector<Consumer*> consumers;
  size_t rr = 0;
  std::vector<Binding> bindings;
  // journal
  int jfd = -1;
  std::string jbuf;
  uint64_t jbytes = 0, live_bytes = 0;
  // counters
  uint64_t published = 0, delivered = 0, acked = 0, redelivered = 0, dead_lettered = 0;
};

struct Pending {
  std::string queue;
  uint64_t msg_id;
};

struct Conn {
  int fd;
  std::string peer, name;
  std::string rbuf, wbuf;
  size_t woff = 0;
  bool closing = false, epollout = false;
  std::map<std::string, std::unique_ptr<Consumer>> consumers;   // queue -> consumer
  std::unordered_map<uint64_t, Pending> unacked;                // delivery tag -> message
  size_t pending_bytes() const { return wbuf.size() - woff; }
};

class Broker {
 public:
  Broker(std::string data_dir, bool fsync_on, uint32_t default_max_redeliv)
      : dir_(std::move(data_dir)), fsync_(fsync_on), default_max_(default_max_redeliv) {}

  bool init(const std::string& host, int port) {
    if (!dir_.empty()) {
      mkdir(dir_.c_str(), 0755);
      load_meta();
    }
    lfd_ = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    if (lfd_ < 0) { perror("socket"); return false; }
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) { fprintf(stderr, "bad host %s\n", host.c_str()); return false; }
    if (bind(lfd_, (sockaddr*)&a, sizeof a) < 0) { perror("bind"); return false; }
    if (listen(lfd_, 256) < 0) { perror("listen"); return false; }
    socklen_t al = sizeof a;
    getsockname(lfd_, (sockaddr*)&a, &al);
    port_ = ntohs(a.sin_port);
    ep_ = epoll_create1(EPOLL_CLOEXEC);
    epoll_event ev{};
    ev.events = EPOLLIN;
    ev.data.ptr = nullptr;
    epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &ev);
    started_ = now_s();
    return true;
  }

  int port() const { return port_; }

  void run() {
    std::vector<epoll_event> evs(256);
    while (!g_stop) {
      int n = epoll_wait(ep_, evs.data(), (int)evs.size(), 500);
      if (n < 0) {
        if (errno == EINTR) continue;
        perror("epoll_wait");
        break;
      }
      for (int i = 0; i < n; ++i) {
        Conn* c = static_cast<Conn*>(evs[i].data.ptr);
        if (c == nullptr) { accept_all(); continue; }
        if (c->closing) continue;
        if (evs[i].events & (EPOLLERR | EPOLLHUP)) { c->closing = true; continue; }
        if (evs[i].events & EPOLLIN) on_readable(c);
        if (!c->closing && (evs[i].events & EPOLLOUT)) flush(c);
      }
      end_of_turn();
    }
    end_of_turn();
    for (auto& kv : queues_) sync_journal(*kv.second, true);
    for (Conn* c : conns_) {
      ::close(c->fd);
      delete c;
    }
    conns_.clear();
    for (auto& kv : queues_)
      if (kv.second->jfd >= 0) ::close(kv.second->jfd);
    if (ep_ >= 0) ::close(ep_);
    if (lfd_ >= 0) ::close(lfd_);
  }

 private:
  // ------------------------------------------------------------ connections
  void accept_all() {
    for (;;) {
      sockaddr_in a{};
      socklen_t al = sizeof a;
      int fd = accept4(lfd_, (sockaddr*)&a, &al, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof one);
      auto* c = new Conn();
      c->fd = fd;
      char buf[64];
      inet_ntop(AF_INET, &a.sin_addr, buf, sizeof buf);
      c->peer = std::string(buf) + ":" + std::to_string(ntohs(a.sin_port));
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.ptr = c;
      epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
      conns_.push_back(c);
    }
  }

  void on_readable(Conn* c) {
    char buf[65536];
    for (;;) {
      ssize_t k = recv(c->fd, buf, sizeof buf, 0);
      if (k > 0) { c->rbuf.append(buf, (size_t)k); continue; }
      if (k == 0) { c->closing = true; break; }
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (errno == EINTR) continue;
      c->closing = true;
      break;
    }
    size_t off = 0;
    while (!c->closing && c->rbuf.size() - off >= 4) {
      const unsigned char* h = reinterpret_cast<const unsigned char*>(c->rbuf.data() + off);
      uint32_t len = ((uint32_t)h[0] << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3];
      if (len == 0 || len > kMaxFrame) { c->closing = true; break; }
      if (c->rbuf.size() - off - 4 < len) break;
      handle(c, (uint8_t)c->rbuf[off + 4], c->rbuf.data() + off + 5, len - 1);
      off += 4 + len;
    }
    c->rbuf.erase(0, off);
  }

  void send(Conn* c, uint8_t op, const std::string& payload) {
    if (c->closing) return;
    c->wbuf.append(frame(op, payload));
    dirty_conns_.push_back(c);
  }

  void flush(Conn* c) {
    const bool was_blocked = c->pending_bytes() > kWriteHighWater;
    while (c->woff < c->wbuf.size()) {
      ssize_t k = ::send(c->fd, c->wbuf.data() + c->woff, c->wbuf.size() - c->woff, MSG_NOSIGNAL);
      if (k > 0) { c->woff += (size_t)k; continue; }
      if (k < 0 && errno == EINTR) continue;
      if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
      c->closing = true;
      return;
    }
    if (c->woff == c->wbuf.size()) { c->wbuf.clear(); c->woff = 0; }
    else if (c->woff > (1u << 20)) { c->wbuf.erase(0, c->woff); c->woff = 0; }
    const bool want = c->woff < c->wbuf.size();
    if (want != c->epollout) {
      epoll_event ev{};
      ev.events = want ? (uint32_t)(EPOLLIN | EPOLLOUT) : (uint32_t)EPOLLIN;
      ev.data.ptr = c;
      epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &ev);
      c->epollout = want;
    }
    // a connection that drained below the high-water mark can take deliveries again
    if (was_blocked && c->pending_bytes() <= kWriteHighWater)
      for (auto& kv : c->consumers) mark_dispatch(kv.first);
  }

  void close_conn(Conn* c) {
    // consumers leave their queues; every unacked delivery goes back to the head of its queue
    for (auto& kv : c->consumers) {
      auto it = queues_.find(kv.first);
      if (it == queues_.end()) continue;
      auto& v = it->second->consumers;
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i] == kv.second.get()) { v.erase(v.begin() + (long)i); break; }
    }
    for (auto& kv : c->unacked) settle(kv.second, /*ack=*/false, /*requeue=*/true);
    epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
    ::close(c->fd);
  }

  // ------------------------------------------------------------ request handling
  void reply_ok(Conn* c, uint32_t req, uint32_t value = 0) {
    Writer w;
    w.u32(req);
    w.u32(value);
    send(c, OP_OK, w.b);
  }
  void reply_err(Conn* c, uint32_t req, const std::string& msg) {
    Writer w;
    w.u32(req);
    w.str(msg);
    send(c, OP_ERR, w.b);
  }

  void handle(Conn* c, uint8_t op, const char* p, size_t n) {
    Reader r(p, n);
    switch (op) {
      case OP_HELLO: {
        uint32_t req = r.u32();
        uint32_t ver = r.u32();
        c->name = r.str();
        if (!r.ok) break;
        if (ver != kProtocolVersion) { reply_err(c, req, "protocol version mismatch"); break; }
        reply_ok(c, req, kProtocolVersion);
        return;
      }
      case OP_PING: {
        uint32_t req = r.u32();
        if (!r.ok) break;
        Writer w;
        w.u32(req);
        send(c, OP_PONG, w.b);
        return;
      }
      case OP_DECLARE: {
        uint32_t req = r.u32();
        std::string q = r.str();
        uint8_t durable = r.u8();
        uint32_t maxr = r.u32();
        if (!r.ok) break;
        if (!valid_name(q)) { reply_err(c, req, "invalid queue name"); return; }
        declare(q, durable != 0, maxr ? maxr : default_max_);
        reply_ok(c, req, (uint32_t)queues_[q]->ready.size());
        return;
      }
      case OP_BIND:
      case OP_UNBIND: {
        uint32_t req = r.u32();
        std::string q = r.str(), ex = r.str(), pat = r.str();
        if (!r.ok) break;
        auto it = queues_.find(q);
        if (it == queues_.end()) { reply_err(c, req, "no such queue: " + q); return; }
        if (!valid_name(ex) || pat.empty() || pat.size() > 255) { reply_err(c, req, "invalid binding"); return; }
        auto& b = it->second->bindings;
        bool found = false;
        for (size_t i = 0; i < b.size(); ++i)
          if (b[i].exchange == ex && b[i].pattern == pat) {
            found = true;
            if (op == OP_UNBIND) b.erase(b.begin() + (long)i);
            break;
          }
        if (op == OP_BIND && !found) b.push_back(Binding{ex, pat, split_words(pat)});
        if (found != (op == OP_BIND)) save_meta();
        reply_ok(c, req);
        return;
      }
      case OP_DELETE: {
        uint32_t req = r.u32();
        std::string q = r.str();
        if (!r.ok) break;
        auto it = queues_.find(q);
        if (it == queues_.end()) { reply_ok(c, req, 0); return; }
        uint32_t dropped = (uint32_t)(it->second->ready.size() + it->second->inflight.size());
        drop_queue(it);
        reply_ok(c, req, dropped);
        return;
      }
      case OP_PURGE: {
        uint32_t req = r.u32();
        std::string q = r.str();
        if (!r.ok) break;
        auto it = queues_.find(q);
        if (it == queues_.end()) { reply_err(c, req, "no such queue: " + q); return; }
        Queue& Q = *it->second;
        uint32_t k = (uint32_t)Q.ready.size();
        for (auto& m : Q.ready) journal_done(Q, m);
        Q.ready.clear();
        reply_ok(c, req, k);
        return;
      }
      case OP_PUBLISH: {
        uint32_t req = r.u32();
        std::string ex = r.str(), rk = r.str();
        std::string body = r.blob();
        if (!r.ok) break;
        uint32_t routed = publish(ex, rk, std::make_shared<const std::string>(std::move(body)));
        confirms_.push_back({c, req, routed});
        return;
      }
      case OP_CONSUME: {
        uint32_t req = r.u32();
        std::string q = r.str();
        uint32_t prefetch = r.u32();
        if (!r.ok) break;
        auto it = queues_.find(q);
        if (it == queues_.end()) { reply_err(c, req, "no such queue: " + q); return; }
        auto& slot = c->consumers[q];
        if (!slot) {
          slot.reset(new Consumer{c, q, prefetch});
          it->second->consumers.push_back(slot.get());
        } else {
          slot->prefetch = prefetch;
        }
        reply_ok(c, req);
        mark_dispatch(q);
        return;
      }
      case OP_CANCEL: {
        uint32_t req = r.u32();
        std::string q = r.str();
        if (!r.ok) break;
        auto ci = c->consumers.find(q);
        if (ci != c->consumers.end()) {
          auto it = queues_.find(q);
          if (it != queues_.end()) {
            auto& v = it->second->consumers;
            for (size_t i = 0; i < v.size(); ++i)
              if (v[i] == ci->second.get()) { v.erase(v.begin() + (long)i); break; }
          }
          // its unacked deliveries stay unacked (acks still count) until the connection closes
          c->consumers.erase(ci);
        }
        reply_ok(c, req);
        return;
      }
      case OP_ACK:
      case OP_NACK: {
        uint64_t tag = r.u64();
        uint8_t requeue = op == OP_NACK ? r.u8() : 0;
        if (!r.ok) break;
        auto it = c->unacked.find(tag);
        if (it == c->unacked.end()) return;   // unknown / already settled: ignore (idempotent)
        Pending pd = it->second;
        c->unacked.erase(it);
        auto ci = c->consumers.find(pd.queue);
        if (ci != c->consumers.end() && ci->second->inflight > 0) ci->second->inflight--;
        settle(pd, op == OP_ACK, requeue != 0);
        mark_dispatch(pd.queue);
        return;
      }
      case OP_GET: {
        uint32_t req = r.u32();
        std::string q = r.str();
        if (!r.ok) break;
        Writer w;
        w.u32(req);
        auto it = queues_.find(q);
        if (it == queues_.end() || it->second->ready.empty()) {
          w.u8(0);
        } else {
          Queue& Q = *it->second;
          Msg m = std::move(Q.ready.front());
          Q.ready.pop_front();
          journal_done(Q, m);
          Q.delivered++;
          Q.acked++;
          w.u8(1);
          w.u32(m.redeliv);
          w.str(m.rk);
          w.blob(*m.body);
        }
        send(c, OP_GET_OK, w.b);
        return;
      }
      case OP_PEEK: {
        uint32_t req = r.u32();
        std::string q = r.str();
        uint32_t limit = r.u32();
        if (!r.ok) break;
        Writer w;
        w.u32(req);
        auto it = queues_.find(q);
        uint32_t k = 0;
        if (it != queues_.end()) k = (uint32_t)std::min<size_t>(limit, it->second->ready.size());
        w.u32(k);
        for (uint32_t i = 0; i < k; ++i) {
          const Msg& m = it->second->ready[i];
          w.u32(m.redeliv);
          w.str(m.rk);
          w.blob(*m.body);
        }
        send(c, OP_PEEK_OK, w.b);
        return;
      }
      case OP_STATS: {
        uint32_t req = r.u32();
        if (!r.ok) break;
        Writer w;
        w.u32(req);
        w.blob(stats_json());
        send(c, OP_STATS_OK, w.b);
        return;
      }
      default:
        break;
    }
    // malformed frame or unknown op: protocol error, drop the connection
    c->closing = true;
  }

  // ------------------------------------------------------------ queues
  Queue& declare(const std::string& q, bool durable, uint32_t maxr) {
    auto it = queues_.find(q);
    if (it != queues_.end()) return *it->second;
    auto Q = std::make_unique<Queue>();
    Q->name = q;
    Q->durable = durable;
    Q->max_redeliv = maxr;
    Queue& ref = *Q;
    queues_[q] = std::move(Q);
    if (durable && !dir_.empty()) open_journal(ref, /*replay=*/true);
    if (!loading_) save_meta();
    return ref;
  }

  void drop_queue(std::map<std::string, std::unique_ptr<Queue>>::iterator it) {
    Queue& Q = *it->second;
    for (Consumer* cs : Q.consumers) cs->conn->consumers.erase(Q.name);
    for (Conn* c : conns_)
      for (auto u = c->unacked.begin(); u != c->unacked.end();)
        u = u->second.queue == Q.name ? c->unacked.erase(u) : std::next(u);
    if (Q.jfd >= 0) {
      ::close(Q.jfd);
      unlink(journal_path(Q.name).c_str());
    }
    queues_.erase(it);
    save_meta();
  }

  uint32_t publish(const std::string& ex, const std::string& rk, std::shared_ptr<const std::string> body) {
    const auto words = split_words(rk);
    uint32_t routed = 0;
    for (auto& kv : queues_) {
      Queue& Q = *kv.second;
      bool hit = false;
      for (auto& b : Q.bindings)
        if (b.exchange == ex && topic_match(b.words, 0, words, 0)) { hit = true; break; }
      if (!hit) continue;
      Msg m;
      m.id = next_id_++;
      m.rk = rk;
      m.body = body;
      journal_enqueue(Q, m);
      Q.ready.push_back(std::move(m));
      Q.published++;
      routed++;
      mark_dispatch(Q.name);
    }
    published_total_++;
    return routed;
  }

  // ack: done.  nack(requeue): back to the head, or to the DLQ past the redelivery limit.
  // nack(no requeue): straight to the DLQ.
  void settle(const Pending& pd, bool ack, bool requeue) {
    auto it = queues_.find(pd.queue);
    if (it == queues_.end()) return;
    Queue& Q = *it->second;
    auto mi = Q.inflight.find(pd.msg_id);
    if (mi == Q.inflight.end()) return;
    Msg m = std::move(mi->second);
    Q.inflight.erase(mi);
    if (ack) {
      Q.acked++;
      journal_done(Q, m);
      return;
    }
    m.redeliv++;
    if (requeue && m.redeliv <= Q.max_redeliv) {
      Q.redelivered++;
      journal_redeliv(Q, m);
      Q.ready.push_front(std::move(m));
      mark_dispatch(Q.name);
      return;
    }
    Q.dead_lettered++;
    journal_done(Q, m);
    if (Q.name.size() > 4 && Q.name.compare(Q.name.size() - 4, 4, ".dlq") == 0) return;   // no DLQ of a DLQ
    const std::string dname = Q.name + ".dlq";
    Queue& D = declare(dname, Q.durable, Q.max_redeliv);
    Msg d;
    d.id = next_id_++;
    d.rk = m.rk;
    d.body = m.body;
    d.redeliv = m.redeliv;
    journal_enqueue(D, d);
    D.ready.push_back(std::move(d));
    D.published++;
    mark_dispatch(dname);
  }

  void mark_dispatch(const std::string& q) { dispatch_.push_back(q); }

  void dispatch(Queue& Q) {
    while (!Q.ready.empty() && !Q.consumers.empty()) {
      Consumer* pick = nullptr;
      for (size_t t = 0; t < Q.consumers.size(); ++t) {
        Consumer* cs = Q.consumers[(Q.rr + t) % Q.consumers.size()];
        if (cs->conn->closing) continue;
        if (cs->prefetch && cs->inflight >= cs->prefetch) continue;
        if (cs->conn->pending_bytes() > kWriteHighWater) continue;
        pick = cs;
        Q.rr = (Q.rr + t + 1) % Q.consumers.size();
        break;
      }
      if (!pick) return;
      Msg m = std::move(Q.ready.front());
      Q.ready.pop_front();
      const uint64_t tag = next_tag_++;
      Writer w;
      w.u64(tag);
      w.u32(m.redeliv);
      w.str(Q.name);
      w.str(m.rk);
      w.blob(*m.body);
      send(pick->conn, OP_DELIVER, w.b);
      pick->inflight++;
      pick->conn->unacked[tag] = Pending{Q.name, m.id};
      Q.delivered++;
      Q.inflight.emplace(m.id, std::move(m));
    }
  }

  void end_of_turn() {
    // 1. durability: journals written + synced before any confirm leaves (group commit)
    for (auto& kv : queues_) sync_journal(*kv.second, false);
    // 2. publisher confirms
    for (auto& cf : confirms_) {
      Writer w;
      w.u32(cf.req);
      w.u32(cf.routed);
      send(cf.c, OP_CONFIRM, w.b);
    }
    confirms_.clear();
    // 3. closed connections: their unacked deliveries go back to the head of their queues
    for (size_t i = 0; i < conns_.size();) {
      Conn* c = conns_[i];
      if (!c->closing) { ++i; continue; }
      close_conn(c);
      std::vector<Conn*> keep;
      for (Conn* d : dirty_conns_) if (d != c) keep.push_back(d);
      dirty_conns_.swap(keep);
      delete c;
      conns_.erase(conns_.begin() + (long)i);
    }
    // 4. deliveries
    while (!dispatch_.empty()) {
      std::vector<std::string> qs;
      qs.swap(dispatch_);
      for (auto& q : qs) {
        auto it = queues_.find(q);
        if (it != queues_.end()) dispatch(*it->second);
      }
    }
    for (auto& kv : queues_) sync_journal(*kv.second, false);
    // 5. socket writes (a connection that fails here is closed on the next turn)
    std::vector<Conn*> dc;
    dc.swap(dirty_conns_);
    for (Conn* c : dc)
      if (!c->closing) flush(c);
  }

  // ------------------------------------------------------------ journal
  // records: 'E' u64 id u32 redeliv str rk blob body | 'D' u64 id | 'R' u64 id u32 redeliv
  std::string journal_path(const std::string& q) const {
    std::string f;
    for (unsigned char ch : q) {
      if (isalnum(ch) || ch == '.' || ch == '_' || ch == '-') f.push_back((char)ch);
      else { char t[4]; snprintf(t, sizeof t, "%%%02X", ch); f.append(t); }
    }
    return dir_ + "/" + f + ".journal";
  }

  static size_t enq_size(const Msg& m) { return 1 + 8 + 4 + 2 + m.rk.size() + 4 + m.body->size(); }

  void journal_enqueue(Queue& Q, const Msg& m) {
    if (Q.jfd < 0) return;
    Writer w;
    w.u8('E');
    w.u64(m.id);
    w.u32(m.redeliv);
    w.str(m.rk);
    w.blob(*m.body);
    Q.jbuf.append(w.b);
    Q.live_bytes += w.b.size();
  }
  void journal_done(Queue& Q, const Msg& m) {
    if (Q.jfd < 0) return;
    Writer w;
    w.u8('D');
    w.u64(m.id);
    Q.jbuf.append(w.b);
    Q.live_bytes -= std::min<uint64_t>(Q.live_bytes, enq_size(m));
  }
  void journal_redeliv(Queue& Q, const Msg& m) {
    if (Q.jfd < 0) return;
    Writer w;
    w.u8('R');
    w.u64(m.id);
    w.u32(m.redeliv);
    Q.jbuf.append(w.b);
  }

  void sync_journal(Queue& Q, bool force) {
    if (Q.jfd < 0 || (Q.jbuf.empty() && !force)) return;
    size_t off = 0;
    while (off < Q.jbuf.size()) {
      ssize_t k = ::write(Q.jfd, Q.jbuf.data() + off, Q.jbuf.size() - off);
      if (k < 0) {
        if (errno == EINTR) continue;
        perror("journal write");
        break;
      }
      off += (size_t)k;
    }
    Q.jbytes += off;
    Q.jbuf.clear();
    if (fsync_) fdatasync(Q.jfd);
    // compaction: rewrite the live messages once the journal is mostly settled records
    if (Q.jbytes > (32u << 20) && Q.live_bytes * 4 < Q.jbytes) compact(Q);
  }

  void compact(Queue& Q) {
    const std::string path = journal_path(Q.name), tmp = path + ".tmp";
    int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return;
    std::vector<const Msg*> all;
    for (auto& m : Q.ready) all.push_back(&m);
    for (auto& kv : Q.inflight) all.push_back(&kv.second);
    Writer w;
    uint64_t live = 0;
    for (const Msg* m : all) {
      size_t before = w.b.size();
      w.u8('E');
      w.u64(m->id);
      w.u32(m->redeliv);
      w.str(m->rk);
      w.blob(*m->body);
      live += w.b.size() - before;
    }
    bool ok = ::write(fd, w.b.data(), w.b.size()) == (ssize_t)w.b.size() && fdatasync(fd) == 0;
    ::close(fd);
    if (!ok || rename(tmp.c_str(), path.c_str()) != 0) { unlink(tmp.c_str()); return; }
    ::close(Q.jfd);
    Q.jfd = ::open(path.c_str(), O_WRONLY | O_APPEND | O_CLOEXEC, 0644);
    Q.jbytes = w.b.size();
    Q.live_bytes = live;
  }

  void open_journal(Queue& Q, bool replay) {
    const std::string path = journal_path(Q.name);
    if (replay) {
      std::string data;
      int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd >= 0) {
        char buf[1 << 16];
        ssize_t k;
        while ((k = ::read(fd, buf, sizeof buf)) > 0) data.append(buf, (size_t)k);
        ::close(fd);
      }
      std::map<uint64_t, Msg> live;
      Reader r(data.data(), data.size());
      size_t good = 0;
      while (r.off < data.size()) {
        uint8_t t = r.u8();
        uint64_t id = r.u64();
        if (t == 'E') {
          Msg m;
          m.id = id;
          m.redeliv = r.u32();
          m.rk = r.str();
          std::string b = r.blob();
          if (!r.ok) break;
          m.body = std::make_shared<const std::string>(std::move(b));
          live[id] = std::move(m);
        } else if (t == 'D') {
          if (!r.ok) break;
          live.erase(id);
        } else if (t == 'R') {
          uint32_t rd = r.u32();
          if (!r.ok) break;
          auto it = live.find(id);
          if (it != live.end()) it->second.redeliv = rd;
        } else {
          r.ok = false;
          break;
        }
        good = r.off;
        if (id >= next_id_) next_id_ = id + 1;
      }
      if (good < data.size()) {
        fprintf(stderr, "cfc-broker: %s: torn tail (%zu bytes) dropped\n", path.c_str(), data.size() - good);
        if (truncate(path.c_str(), (off_t)good) != 0) perror("truncate");
      }
      for (auto& kv : live) {
        Q.live_bytes += enq_size(kv.second);
        Q.ready.push_back(std::move(kv.second));
      }
      Q.jbytes = good;
    }
    Q.jfd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (Q.jfd < 0) perror("journal open");
  }

  // queues + bindings: "Q\t<durable>\t<max>\t<name>" / "B\t<queue>\t<exchange>\t<pattern>"
  void save_meta() {
    if (dir_.empty()) return;
    std::string s;
    for (auto& kv : queues_) {
      const Queue& Q = *kv.second;
      if (!Q.durable) continue;
      s += "Q\t" + std::to_string(Q.durable ? 1 : 0) + "\t" + std::to_string(Q.max_redeliv) + "\t" + Q.name + "\n";
      for (auto& b : Q.bindings) s += "B\t" + Q.name + "\t" + b.exchange + "\t" + b.pattern + "\n";
    }
    const std::string path = dir_ + "/meta.tsv", tmp = path + ".tmp";
    int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return;
    bool ok = ::write(fd, s.data(), s.size()) == (ssize_t)s.size();
    if (fsync_) fdatasync(fd);
    ::close(fd);
    if (ok) rename(tmp.c_str(), path.c_str());
  }

  void load_meta() {
    FILE* f = fopen((dir_ + "/meta.tsv").c_str(), "r");
    if (!f) return;
    char line[2048];
    std::vector<std::vector<std::string>> rows;
    while (fgets(line, sizeof line, f)) {
      std::string s(line);
      while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
      std::vector<std::string> parts;
      size_t a = 0;
      for (;;) {
        size_t b = s.find('\t', a);
        parts.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) break;
        a = b + 1;
      }
      rows.push_back(parts);
    }
    fclose(f);
    loading_ = true;
    for (auto& p : rows)
      if (p.size() == 4 && p[0] == "Q" && valid_name(p[3]))
        declare(p[3], p[1] == "1", (uint32_t)strtoul(p[2].c_str(), nullptr, 10));
    for (auto& p : rows)
      if (p.size() == 4 && p[0] == "B") {
        auto it = queues_.find(p[1]);
        if (it != queues_.end()) it->second->bindings.push_back(Binding{p[2], p[3], split_words(p[3])});
      }
    loading_ = false;
  }

  std::string stats_json() const {
    std::string s = "{\"uptime_s\": " + std::to_string(now_s() - started_) +
                    ", \"connections\": " + std::to_string(conns_.size()) +
                    ", \"published\": " + std::to_string(published_total_) + ", \"queues\": {";
    bool first = true;
    for (auto& kv : queues_) {
      const Queue& Q = *kv.second;
      if (!first) s += ", ";
      first = false;
      s += "\"" + json_escape(Q.name) + "\": {\"ready\": " + std::to_string(Q.ready.size()) +
           ", \"unacked\": " + std::to_string(Q.inflight.size()) +
           ", \"consumers\": " + std::to_string(Q.consumers.size()) +
           ", \"durable\": " + (Q.durable ? "true" : "false") +
           ", \"max_redeliveries\": " + std::to_string(Q.max_redeliv) +
           ", \"published\": " + std::to_string(Q.published) +
           ", \"delivered\": " + std::to_string(Q.delivered) + ", \"acked\": " + std::to_string(Q.acked) +
           ", \"redelivered\": " + std::to_string(Q.redelivered) +
           ", \"dead_lettered\": " + std::to_string(Q.dead_lettered) +
           ", \"journal_bytes\": " + std::to_string(Q.jbytes) + ", \"bindings\": [";
      for (size_t i = 0; i < Q.bindings.size(); ++i) {
        if (i) s += ", ";
        s += "[\"" + json_escape(Q.bindings[i].exchange) + "\", \"" + json_escape(Q.bindings[i].pattern) + "\"]";
      }
      s += "]}";
    }
    return s + "}}";
  }

  struct Confirm {
    Conn* c;
    uint32_t req, routed;
  };

  std::string dir_;
  bool fsync_;
  uint32_t default_max_;
  bool loading_ = false;
  int lfd_ = -1, ep_ = -1, port_ = 0;
  double started_ = 0;
  uint64_t next_id_ = 1, next_tag_ = 1, published_total_ = 0;
  std::map<std::string, std::unique_ptr<Queue>> queues_;
  std::vector<Conn*> conns_, dirty_conns_;
  std::vector<std::string> dispatch_;
  std::vector<Confirm> confirms_;
};

void usage() {
  fprintf(stderr,
          "usage: cfc-broker [--host 0.0.0.0] [--port 5680] [--data-dir DIR] [--fsync always|never]\n"
          "                  [--max-redeliveries 5]\n"
          "  --port 0 picks a free port; the chosen port is printed as 'cfc-broker listening on HOST:PORT'.\n"
          "  Without --data-dir nothing is persisted (every queue behaves as transient).\n");
}

}  // namespace

int main(int argc, char** argv) {
  std::string host = "0.0.0.0", dir;
  int port = 5680;
  bool fsync_on = true;
  uint32_t maxr = 5;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) { usage(); exit(2); }
      return argv[++i];
    };
    if (a == "--host") host = val();
    else if (a == "--port") port = atoi(val().c_str());
    else if (a == "--data-dir") dir = val();
    else if (a == "--fsync") fsync_on = val() != "never";
    else if (a == "--max-redeliveries") maxr = (uint32_t)strtoul(val().c_str(), nullptr, 10);
    else if (a == "-h" || a == "--help") { usage(); return 0; }
    else { usage(); return 2; }
  }
  struct sigaction sa {};
  sa.sa_handler = on_signal;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  signal(SIGPIPE, SIG_IGN);
  Broker b(dir, fsync_on, maxr);
  if (!b.init(host, port)) return 1;
  printf("cfc-broker listening on %s:%d\n", host.c_str(), b.port());
  fflush(stdout);
  b.run();
  return 0;
}
