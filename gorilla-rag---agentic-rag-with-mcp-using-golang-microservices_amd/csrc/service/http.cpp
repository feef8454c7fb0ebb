// http.cpp — the HTTP/1.1 listener in front of the handler mirror
// (include/vsearch_service.h vsvc_http_*), and the framing the load
// generator's TCP mode uses as a client.
//
// The reference serves its four routes with net/http
// (rag/vector-service/main.go:70-77: http.HandleFunc on the default mux,
// http.ListenAndServe(":"+PORT)); retrieval-service reaches it with
// http.Post (rag/retrieval-service/main.go:229-233). This listener keeps
// the net/http behaviour those callers see: HTTP/1.1 keep-alive (and
// pipelined requests, answered in order), Content-Length and chunked request
// bodies, `Expect: 100-continue`, HEAD, TCP_NODELAY, the mux matching the
// URL path without its query, a 400 for a malformed request or a missing
// Host header, 431 past 1 MiB of headers (DefaultMaxHeaderBytes), 501 for a
// transfer coding other than chunked, 505 for a version other than 1.x.
// One thread per connection stands in for net/http's goroutine per
// connection; every request goes to vsvc_handle (thread-safe), so concurrent
// /search requests meet in the batcher exactly as in-process calls do.
#include "http.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <list>
#include <memory>
#include <mutex>
#include <thread>

#include "../../../include/vsearch_service.h"

namespace vshttp {

namespace {

bool ieq(const std::string& a, const char* b) {
  const size_t n = std::strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; ++i)
    if (std::tolower((unsigned char)a[i]) != std::tolower((unsigned char)b[i])) return false;
  return true;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) --b;
  return s.substr(a, b - a);
}

bool is_tchar(char c) {
  return std::isalnum((unsigned char)c) || std::strchr("!#$%&'*+-.^_`|~", c) != nullptr;
}

// Finds the end of a message head: the index just past the blank line that
// ends it ("\r\n\r\n", or bare "\n" line ends as textproto accepts), or npos.
size_t head_end(const char* b, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    if (b[i] != '\n') continue;
    if (i + 1 < n && b[i + 1] == '\n') return i + 2;
    if (i + 2 < n && b[i + 1] == '\r' && b[i + 2] == '\n') return i + 3;
  }
  return std::string::npos;
}

// Splits a head into lines without their line ends (the blank line dropped).
void head_lines(const char* b, size_t n, std::string* first, std::list<std::string>* lines) {
  size_t s = 0;
  bool got_first = false;
  for (size_t i = 0; i < n; ++i) {
    if (b[i] != '\n') continue;
    size_t e = i;
    if (e > s && b[e - 1] == '\r') --e;
    if (e > s || got_first) {
      std::string ln(b + s, e - s);
      if (!got_first) {
        *first = std::move(ln);
        got_first = true;
      } else if (!ln.empty()) {
        lines->push_back(std::move(ln));
      }
    }
    s = i + 1;
  }
}

bool parse_digits(const std::string& v, int64_t* out) {
  if (v.empty() || v.size() > 18) return false;
  int64_t x = 0;
  for (char c : v) {
    if (c < '0' || c > '9') return false;
    x = x * 10 + (c - '0');
  }
  *out = x;
  return true;
}

// Comma-separated header tokens (Connection), lower-cased.
bool has_token(const std::string& v, const char* tok) {
  size_t s = 0;
  while (s <= v.size()) {
    size_t e = v.find(',', s);
    if (e == std::string::npos) e = v.size();
    if (ieq(trim(v.substr(s, e - s)), tok)) return true;
    s = e + 1;
  }
  return false;
}

}  // namespace

const char* status_text(int s) {
  switch (s) {
    case 100: return "Continue";
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 408: return "Request Timeout";
    case 411: return "Length Required";
    case 413: return "Request Entity Too Large";
    case 417: return "Expectation Failed";
    case 431: return "Request Header Fields Too Large";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 503: return "Service Unavailable";
    case 505: return "HTTP Version Not Supported";
    default: return "";
  }
}

Frame parse_request_head(const char* buf, size_t len, Request* req, size_t* head_len,
                         int* bad_status) {
  const size_t he = head_end(buf, len);
  if (he == std::string::npos) {
    if (len > kMaxHeaderBytes) {
      *bad_status = 431;
      return Frame::kBad;
    }
    return Frame::kNeedMore;
  }
  if (he > kMaxHeaderBytes + 4) {
    *bad_status = 431;
    return Frame::kBad;
  }
  *bad_status = 400;
  std::string first;
  std::list<std::string> lines;
  head_lines(buf, he, &first, &lines);
  // request line: METHOD SP target SP HTTP/1.x
  const size_t s1 = first.find(' ');
  const size_t s2 = s1 == std::string::npos ? s1 : first.find(' ', s1 + 1);
  if (s1 == std::string::npos || s2 == std::string::npos || s1 == 0 || s2 == s1 + 1)
    return Frame::kBad;
  req->method = first.substr(0, s1);
  req->target = first.substr(s1 + 1, s2 - s1 - 1);
  const std::string ver = first.substr(s2 + 1);
  for (char c : req->method)
    if (!is_tchar(c)) return Frame::kBad;
  if (req->target.find(' ') != std::string::npos) return Frame::kBad;
  if (ver.size() != 8 || ver.compare(0, 5, "HTTP/") != 0 || ver[6] != '.' ||
      !std::isdigit((unsigned char)ver[5]) || !std::isdigit((unsigned char)ver[7]))
    return Frame::kBad;
  if (ver[5] != '1') {
    *bad_status = 505;
    return Frame::kBad;
  }
  req->minor = ver[7] - '0';
  req->keep_alive = req->minor >= 1;
  req->expect_continue = false;
  req->chunked = false;
  req->content_length = -1;
  bool have_host = false, saw_te = false;
  for (const std::string& ln : lines) {
    if (ln[0] == ' ' || ln[0] == '\t') return Frame::kBad;  // obsolete line folding
    const size_t c = ln.find(':');
    if (c == std::string::npos || c == 0) return Frame::kBad;
    const std::string name = ln.substr(0, c);
    for (char ch : name)
      if (!is_tchar(ch)) return Frame::kBad;
    const std::string v = trim(ln.substr(c + 1));
    if (ieq(name, "content-length")) {
      int64_t cl;
      if (!parse_digits(v, &cl)) return Frame::kBad;
      if (req->content_length >= 0 && req->content_length != cl) return Frame::kBad;
      req->content_length = cl;
    } else if (ieq(name, "transfer-encoding")) {
      // net/http: exactly one Transfer-Encoding line, and it must be
      // "chunked" ("too many transfer encodings" / "unsupported transfer
      // encoding" -> 501); a second line is ambiguous framing
      if (saw_te || !ieq(v, "chunked")) {
        *bad_status = 501;
        return Frame::kBad;
      }
      saw_te = true;
      req->chunked = true;
    } else if (ieq(name, "connection")) {
      if (has_token(v, "close")) req->keep_alive = false;
      else if (req->minor == 0 && has_token(v, "keep-alive")) req->keep_alive = true;
    } else if (ieq(name, "expect")) {
      if (ieq(v, "100-continue")) {
        req->expect_continue = true;
      } else if (!v.empty()) {
        *bad_status = 417;
        return Frame::kBad;
      }
    } else if (ieq(name, "host")) {
      have_host = true;
    }
  }
  if (req->minor >= 1 && !have_host) return Frame::kBad;  // "missing required Host header"
  if (req->chunked) req->content_length = -1;            // chunked wins (RFC 7230 3.3.3)
  if (req->content_length > kMaxBodyBytes) {
    *bad_status = 413;
    return Frame::kBad;
  }
  // the mux matches URL.Path: drop an absolute-form prefix and the query
  std::string p = req->target;
  if (p.compare(0, 7, "http://") == 0 || p.compare(0, 8, "https://") == 0) {
    const size_t sl = p.find('/', p.find("//") + 2);
    p = sl == std::string::npos ? "/" : p.substr(sl);
  }
  const size_t q = p.find_first_of("?#");
  if (q != std::string::npos) p.resize(q);
  req->path = p;
  *head_len = he;
  return Frame::kDone;
}

Frame body_frame(const char* buf, size_t len, bool chunked, int64_t content_length,
                 std::string* body, size_t* consumed, ChunkScan* scan) {
  if (!chunked) {
    const size_t cl = content_length > 0 ? (size_t)content_length : 0;
    if (len < cl) return Frame::kNeedMore;
    body->assign(buf, cl);
    *consumed = cl;
    return Frame::kDone;
  }
  // framing first (chunks already framed by an earlier call are skipped,
  // and chunk data is jumped over), then one copy of the data
  ChunkScan local;
  ChunkScan& st = scan ? *scan : local;
  size_t pos = st.pos;
  while (!st.in_trailer) {
    const void* nl = std::memchr(buf + pos, '\n', len - pos);
    if (!nl) return len - pos > 4096 ? Frame::kBad : Frame::kNeedMore;
    const size_t e = (const char*)nl - buf;
    size_t x = pos;
    uint64_t sz = 0;
    int nd = 0;
    for (; x < e; ++x) {
      const char c = buf[x];
      const int v = c >= '0' && c <= '9' ? c - '0'
                    : (c >= 'a' && c <= 'f' ? c - 'a' + 10 : (c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1));
      if (v < 0) break;
      if (++nd > 15) return Frame::kBad;
      sz = sz * 16 + (uint64_t)v;
    }
    if (nd == 0) return Frame::kBad;
    // chunk extensions (";name=value") and the CR are ignored
    if (x < e && buf[x] != ';' && buf[x] != '\r' && buf[x] != ' ' && buf[x] != '\t')
      return Frame::kBad;
    size_t p = e + 1;
    if (sz == 0) {
      // the last chunk: the trailer section follows (resumable below)
      st.in_trailer = true;
      st.pos = pos = p;
      break;
    }
    if ((int64_t)(st.total + sz) > kMaxBodyBytes) return Frame::kBad;
    if (len - p < sz + 1) return Frame::kNeedMore;
    const size_t data = p;
    p += sz;
    if (buf[p] == '\r') {
      if (len - p < 2) return Frame::kNeedMore;
      if (buf[p + 1] != '\n') return Frame::kBad;
      p += 2;
    } else if (buf[p] == '\n') {
      p += 1;
    } else {
      return Frame::kBad;
    }
    // this chunk is complete: record it and resume after it next time
    st.parts.emplace_back(data, (size_t)sz);
    st.total += sz;
    st.pos = pos = p;
  }
  // trailer section: header lines up to a blank line, counted against the
  // header limit; every complete line is recorded, so a slow trailer is not
  // rescanned from the start on each receive
  for (;;) {
    const void* tl = std::memchr(buf + pos, '\n', len - pos);
    if (!tl) {
      if (st.trailer_bytes + (len - pos) > kMaxHeaderBytes) return Frame::kBad;
      return Frame::kNeedMore;
    }
    const size_t te = (const char*)tl - buf;
    const bool blank = te == pos || (te == pos + 1 && buf[pos] == '\r');
    st.trailer_bytes += te + 1 - pos;
    if (st.trailer_bytes > kMaxHeaderBytes) return Frame::kBad;
    st.pos = pos = te + 1;
    if (blank) break;
  }
  body->clear();
  body->reserve(st.total);
  for (const auto& pr : st.parts) body->append(buf + pr.first, pr.second);
  *consumed = pos;
  return Frame::kDone;
}

Frame parse_response(const char* buf, size_t len, Response* resp, size_t* consumed) {
  const size_t he = head_end(buf, len);
  if (he == std::string::npos) return len > kMaxHeaderBytes ? Frame::kBad : Frame::kNeedMore;
  std::string first;
  std::list<std::string> lines;
  head_lines(buf, he, &first, &lines);
  // HTTP/1.x SP 3DIGIT [SP reason]
  if (first.size() < 12 || first.compare(0, 7, "HTTP/1.") != 0 || first[8] != ' ')
    return Frame::kBad;
  int64_t st = 0;
  if (!parse_digits(first.substr(9, 3), &st)) return Frame::kBad;
  resp->status = (int)st;
  resp->keep_alive = first[7] != '0';
  resp->content_type.clear();
  int64_t cl = -1;
  bool chunked = false;
  for (const std::string& ln : lines) {
    const size_t c = ln.find(':');
    if (c == std::string::npos) return Frame::kBad;
    const std::string name = ln.substr(0, c), v = trim(ln.substr(c + 1));
    if (ieq(name, "content-length")) {
      if (!parse_digits(v, &cl)) return Frame::kBad;
    } else if (ieq(name, "transfer-encoding")) {
      chunked = ieq(v, "chunked");
    } else if (ieq(name, "connection")) {
      if (has_token(v, "close")) resp->keep_alive = false;
      else if (has_token(v, "keep-alive")) resp->keep_alive = true;
    } else if (ieq(name, "content-type")) {
      resp->content_type = v;
    }
  }
  if ((st >= 100 && st < 200) || st == 204 || st == 304) {
    resp->body.clear();
    *consumed = he;
    return Frame::kDone;
  }
  if (!chunked && cl < 0) {
    // body delimited by the close: not produced by this server
    resp->keep_alive = false;
    cl = 0;
  }
  size_t bc = 0;
  const Frame f = body_frame(buf + he, len - he, chunked, cl, &resp->body, &bc);
  if (f == Frame::kDone) *consumed = he + bc;
  return f;
}

std::string response_head(int status, const char* content_type, size_t body_len, bool close,
                          bool keep_alive_10) {
  static const char* kDay[] = {"Sun", "Mon", "Tue", "Wed", "Thu", "Fri", "Sat"};
  static const char* kMon[] = {"Jan", "Feb", "Mar", "Apr", "May", "Jun",
                               "Jul", "Aug", "Sep", "Oct", "Nov", "Dec"};
  const time_t now = time(nullptr);
  struct tm g;
  gmtime_r(&now, &g);
  char date[64];
  std::snprintf(date, sizeof(date), "%s, %02d %s %04d %02d:%02d:%02d GMT", kDay[g.tm_wday % 7],
                g.tm_mday, kMon[g.tm_mon % 12], g.tm_year + 1900, g.tm_hour, g.tm_min, g.tm_sec);
  std::string h;
  h.reserve(192);
  h += "HTTP/1.1 ";
  h += std::to_string(status);
  h += ' ';
  h += status_text(status);
  h += "\r\n";
  if (content_type) {
    h += "Content-Type: ";
    h += content_type;
    h += "\r\n";
    // http.Error sets it beside its text/plain body
    if (std::strncmp(content_type, "text/plain", 10) == 0) h += "X-Content-Type-Options: nosniff\r\n";
  }
  h += "Date: ";
  h += date;
  h += "\r\nContent-Length: ";
  h += std::to_string(body_len);
  h += "\r\n";
  if (close) h += "Connection: close\r\n";
  if (keep_alive_10) h += "Connection: keep-alive\r\n";  // an HTTP/1.0 client asked for it
  h += "\r\n";
  return h;
}

bool send_all(int fd, const char* p, size_t n) {
  while (n) {
    const ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

bool recv_some(int fd, std::string* buf) {
  char tmp[65536];
  for (;;) {
    const ssize_t r = ::recv(fd, tmp, sizeof(tmp), 0);
    if (r > 0) {
      buf->append(tmp, (size_t)r);
      return true;
    }
    if (r < 0 && errno == EINTR) continue;
    return false;
  }
}

int connect_tcp(const std::string& host, int port) {
  struct addrinfo hints, *res = nullptr;
  std::memset(&hints, 0, sizeof(hints));
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  const std::string h = host.empty() ? std::string("127.0.0.1") : host;
  if (::getaddrinfo(h.c_str(), std::to_string(port).c_str(), &hints, &res) != 0 || !res) return -1;
  int fd = ::socket(res->ai_family, res->ai_socktype | SOCK_CLOEXEC, res->ai_protocol);
  if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
    ::close(fd);
    fd = -1;
  }
  ::freeaddrinfo(res);
  if (fd >= 0) {
    const int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  return fd;
}

bool split_addr(const std::string& addr, std::string* host, int* port) {
  const size_t c = addr.rfind(':');
  if (c == std::string::npos) return false;
  int64_t p;
  if (!parse_digits(addr.substr(c + 1), &p) || p > 65535) return false;
  *host = addr.substr(0, c);
  *port = (int)p;
  return true;
}

}  // namespace vshttp

// ---------------------------------------------------------------------------
// the listener
// ---------------------------------------------------------------------------

namespace {

using vshttp::Frame;

// One connection: its thread, its socket (closed only by whoever joins the
// thread, so a shutdown() from vsvc_http_stop never reaches a reused fd).
struct ConnSlot {
  int fd = -1;
  std::thread th;
  std::atomic<bool> done{false};
};

constexpr size_t kMaxConns = 4096;

void send_error_close(int fd, int status) {
  // net/http answers a malformed request with "<code> <text>" and closes
  std::string body = std::to_string(status) + " " + vshttp::status_text(status);
  const std::string h = vshttp::response_head(status, "text/plain; charset=utf-8", body.size(), true);
  vshttp::send_all(fd, h.data(), h.size());
  vshttp::send_all(fd, body.data(), body.size());
}

void serve_conn(vsvc* svc, ConnSlot* cs, const std::atomic<bool>* stop) {
  const int fd = cs->fd;
  std::string buf;
  size_t off = 0;
  vshttp::Request req;
  while (!stop->load(std::memory_order_relaxed)) {
    if (off == buf.size()) {
      buf.clear();
      off = 0;
    } else if (off > (1u << 20)) {
      buf.erase(0, off);
      off = 0;
    }
    size_t hl = 0;
    int bad = 400;
    const Frame f = vshttp::parse_request_head(buf.data() + off, buf.size() - off, &req, &hl, &bad);
    if (f == Frame::kNeedMore) {
      if (!vshttp::recv_some(fd, &buf)) break;
      continue;
    }
    if (f == Frame::kBad) {
      send_error_close(fd, bad);
      break;
    }
    off += hl;
    // room for the announced body, up to 64 MiB ahead (a larger one grows as
    // it arrives: a header alone never commits gigabytes)
    if (req.content_length > 0)
      buf.reserve(off + std::min<size_t>((size_t)req.content_length, size_t(64) << 20));
    bool sent_continue = false, ok = true;
    size_t used = 0;
    vshttp::ChunkScan cscan;
    for (;;) {
      const Frame b = vshttp::body_frame(buf.data() + off, buf.size() - off, req.chunked,
                                         req.content_length, &req.body, &used, &cscan);
      if (b == Frame::kDone) break;
      if (b == Frame::kBad) {
        send_error_close(fd, 400);
        ok = false;
        break;
      }
      if (req.expect_continue && !sent_continue) {
        static const char k100[] = "HTTP/1.1 100 Continue\r\n\r\n";
        if (!vshttp::send_all(fd, k100, sizeof(k100) - 1)) {
          ok = false;
          break;
        }
        sent_continue = true;
      }
      if (!vshttp::recv_some(fd, &buf)) {
        ok = false;
        break;
      }
    }
    if (!ok) break;
    off += used;
    const bool head = req.method == "HEAD";
    int status = 500;
    char* resp = nullptr;
    size_t rlen = 0;
    const char* ct = nullptr;
    const int rc = vsvc_handle(svc, head ? "GET" : req.method.c_str(), req.path.c_str(),
                               req.body.data(), req.body.size(), &status, &resp, &rlen, &ct);
    if (rc != VS_OK || !resp) {
      vsvc_free(resp);
      send_error_close(fd, 500);
      break;
    }
    std::string out = vshttp::response_head(status, ct, rlen, !req.keep_alive,
                                            req.minor == 0 && req.keep_alive);
    if (!head) out.append(resp, rlen);
    vsvc_free(resp);
    req.body.clear();
    if (!vshttp::send_all(fd, out.data(), out.size())) break;
    if (!req.keep_alive) break;
  }
  ::shutdown(fd, SHUT_RDWR);
  cs->done.store(true, std::memory_order_release);
}

}  // namespace

struct vsvc_http {
  vsvc* svc = nullptr;
  int lfd = -1;
  int wake[2] = {-1, -1};
  int port = 0;
  std::atomic<bool> stop{false};
  std::thread acceptor;
  std::mutex mu;
  std::list<std::unique_ptr<ConnSlot>> conns;

  // joins and closes finished connections (acceptor thread / stop)
  void reap(bool all) {
    std::list<std::unique_ptr<ConnSlot>> fin;
    {
      std::lock_guard<std::mutex> g(mu);
      for (auto it = conns.begin(); it != conns.end();) {
        if (all || (*it)->done.load(std::memory_order_acquire)) {
          fin.push_back(std::move(*it));
          it = conns.erase(it);
        } else {
          ++it;
        }
      }
    }
    for (auto& c : fin) {
      if (c->th.joinable()) c->th.join();
      ::close(c->fd);
    }
  }

  void accept_loop() {
    for (;;) {
      struct pollfd p[2] = {{lfd, POLLIN, 0}, {wake[0], POLLIN, 0}};
      const int r = ::poll(p, 2, 1000);
      if (stop.load()) break;
      reap(false);
      if (r <= 0 || !(p[0].revents & POLLIN)) continue;
      const int fd = ::accept4(lfd, nullptr, nullptr, SOCK_CLOEXEC);
      if (fd < 0) continue;
      const int one = 1;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));  // net/http's default
      // recv gives up after kIdleTimeoutSec without a byte: the connection closes
      struct timeval tv = {vshttp::kIdleTimeoutSec, 0};
      ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
      std::lock_guard<std::mutex> g(mu);
      if (conns.size() >= kMaxConns) {
        send_error_close(fd, 503);
        ::close(fd);
        continue;
      }
      auto cs = std::make_unique<ConnSlot>();
      cs->fd = fd;
      ConnSlot* raw = cs.get();
      conns.push_back(std::move(cs));
      raw->th = std::thread(serve_conn, svc, raw, &stop);
    }
  }
};

extern "C" {

int vsvc_http_start(vsvc* svc, const char* addr, vsvc_http** out) {
  if (!svc || !addr || !out) return VS_ERR_INVALID_ARG;
  *out = nullptr;
  std::string host;
  int port = 0;
  if (!vshttp::split_addr(addr, &host, &port)) return VS_ERR_INVALID_ARG;
  struct sockaddr_in sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (host.empty() || host == "0.0.0.0") {
    sa.sin_addr.s_addr = htonl(INADDR_ANY);
  } else {
    if (host == "localhost") host = "127.0.0.1";
    if (::inet_pton(AF_INET, host.c_str(), &sa.sin_addr) != 1) return VS_ERR_INVALID_ARG;
  }
  const int lfd = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd < 0) return VS_ERR_IO;
  const int one = 1;
  ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (::bind(lfd, (struct sockaddr*)&sa, sizeof(sa)) != 0 || ::listen(lfd, 1024) != 0) {
    ::close(lfd);
    return VS_ERR_IO;
  }
  socklen_t sl = sizeof(sa);
  ::getsockname(lfd, (struct sockaddr*)&sa, &sl);
  auto h = std::make_unique<vsvc_http>();
  h->svc = svc;
  h->lfd = lfd;
  h->port = ntohs(sa.sin_port);
  if (::pipe2(h->wake, O_CLOEXEC) != 0) {
    ::close(lfd);
    return VS_ERR_IO;
  }
  vsvc_http* raw = h.get();
  raw->acceptor = std::thread([raw] { raw->accept_loop(); });
  *out = h.release();
  return VS_OK;
}

int vsvc_http_port(const vsvc_http* h) { return h ? h->port : -1; }

void vsvc_http_stop(vsvc_http* h) {
  if (!h) return;
  h->stop.store(true);
  const char c = 1;
  if (::write(h->wake[1], &c, 1) < 0) { /* the 1 s poll timeout wakes it anyway */ }
  if (h->acceptor.joinable()) h->acceptor.join();
  ::close(h->lfd);
  {
    // wake connection threads blocked in recv (idle keep-alive connections)
    std::lock_guard<std::mutex> g(h->mu);
    for (auto& c : h->conns) ::shutdown(c->fd, SHUT_RDWR);
  }
  h->reap(true);
  ::close(h->wake[0]);
  ::close(h->wake[1]);
  delete h;
}

}  // extern "C"
