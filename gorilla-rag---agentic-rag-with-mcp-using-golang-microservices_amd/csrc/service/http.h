// http.h — HTTP/1.1 message framing shared by the listener (vsvc_http_start)
// and the load generator's TCP mode. Internal to the service library.
#ifndef VS_SERVICE_HTTP_H_
#define VS_SERVICE_HTTP_H_

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace vshttp {

// Outcome of framing one message out of a receive buffer.
enum class Frame { kNeedMore, kDone, kBad };

// One parsed request (net/http's Request, the parts the handlers read).
struct Request {
  std::string method, target, path;  // path: target without query / absolute-form prefix
  int minor = 1;                     // HTTP/1.<minor>
  bool keep_alive = true;
  bool expect_continue = false;
  bool chunked = false;
  int64_t content_length = -1;  // -1: none given
  std::string body;
};

// One parsed response (the client side of the load generator).
struct Response {
  int status = 0;
  bool keep_alive = true;
  std::string content_type;
  std::string body;
};

constexpr size_t kMaxHeaderBytes = 1 << 20;  // net/http DefaultMaxHeaderBytes
// Request bodies past this are refused (413 by Content-Length, 400 for a
// chunked body that grows past it). A /search body is ~16 KB and an ingest
// upsert batch a few MB; net/http itself sets no limit.
constexpr int64_t kMaxBodyBytes = int64_t(256) << 20;
// A connection that sends nothing for this long (idle keep-alive, or a
// stalled request) is closed, like net/http's Server.IdleTimeout would.
constexpr int kIdleTimeoutSec = 120;

// Parses the request head in buf[0, ...). On kDone, *head_len is the byte
// count of the head (through the blank line) and req's head fields are set.
// On kBad, *bad_status is the status to answer with (400, 413, 417, 431, 501,
// 505) before closing. Bodies are framed by body_frame below.
Frame parse_request_head(const char* buf, size_t len, Request* req, size_t* head_len,
                         int* bad_status);

// Progress of framing one chunked body across calls (bytes arrive in
// pieces): the chunks already framed are not scanned again.
struct ChunkScan {
  size_t pos = 0;    // offset of the next chunk-size line (or trailer line)
  size_t total = 0;  // data bytes framed so far
  std::vector<std::pair<size_t, size_t>> parts;  // (offset, length) of each chunk's data
  bool in_trailer = false;  // the 0-size chunk was framed; pos walks the trailer lines
  size_t trailer_bytes = 0; // trailer bytes framed so far (capped at kMaxHeaderBytes)
};

// Frames a body that starts at buf[0]: Content-Length or chunked (trailers
// skipped). On kDone, *consumed is the byte count of the framed body and
// *body the decoded bytes. kBad: malformed chunk framing, a body past
// kMaxBodyBytes or a trailer past kMaxHeaderBytes. `scan` (chunked
// only; nullable) carries the progress between calls on a growing buffer;
// reset it for every new body.
Frame body_frame(const char* buf, size_t len, bool chunked, int64_t content_length,
                 std::string* body, size_t* consumed, ChunkScan* scan = nullptr);

// Parses a response head + body (Content-Length, chunked, or none for 1xx /
// 204 / 304). On kDone, *consumed is the byte count of the whole message.
Frame parse_response(const char* buf, size_t len, Response* resp, size_t* consumed);

// The reason phrase net/http's StatusText gives for a status.
const char* status_text(int status);

// Serialises a response head: status line, Content-Type, Date, Content-Length
// and, for text/plain bodies (http.Error), X-Content-Type-Options: nosniff.
// keep_alive_10: an HTTP/1.0 request asked to keep the connection
// ("Connection: keep-alive" is echoed, as net/http does).
std::string response_head(int status, const char* content_type, size_t body_len, bool close,
                          bool keep_alive_10 = false);

// Blocking helpers over a connected socket. send_all uses MSG_NOSIGNAL.
bool send_all(int fd, const char* p, size_t n);
// Appends what recv returns; false on EOF or error.
bool recv_some(int fd, std::string* buf);

// Connects a TCP socket to host:port (IPv4 literal or a name getaddrinfo
// resolves) with TCP_NODELAY; -1 on failure.
int connect_tcp(const std::string& host, int port);

// Splits "host:port" (":8082" -> listen on every address; "[::1]:80" form
// not supported). false on a malformed address.
bool split_addr(const std::string& addr, std::string* host, int* port);

}  // namespace vshttp

#endif  // VS_SERVICE_HTTP_H_
