// remote_ui.hpp -- the render server's remote-UI hooks, built
// into bin/splat when REMOTE_UI=1 (the default; Makefile).
//
// Mirrors include/remote_ui/InterfaceServer.hpp and AsyncTask.hpp of the
// reference: a server thread accepts one TCP client, both sides exchange
// "ready", client packets update a State (InterfaceServer.hpp:230-244) that
// the render loop consumes once per frame (consumeState, :247-251), and the
// server sends the tile histogram (sendHistogram, :330-332), a preview image
// of every frame (sendPreviewImage, :322-328) and the fov (updateFov,
// :302-307).
//
// The reference's transport libraries (packetcomms, videolib: empty
// submodules in the snapshot) are not available, so the wire format is this
// build's own, with the reference's packet names and their order
// (InterfaceServer.hpp:24-43):
//   packet  = u32 type (index in kPacketTypes) | u32 payload bytes | payload
//   float   = f32; bool = u8; string = u64 length | bytes;
//   vector<u32> = u64 count | u32 x count      (cereal's binary layout)
//   render_preview = i32 width | i32 height | u32 codec (1: zlib BGR24) | data
// The preview is a zlib-compressed BGR24 frame instead of an FFmpeg stream.
// A client that disconnects without "stop" also stops the server's loop (the
// reference keeps rendering with nobody attached).
#pragma once

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace gsui {

const std::vector<std::string> kPacketTypes{
    "stop", "detach", "env_rotation", "env_rotation_2", "exposure", "gamma", "X", "Y", "Z",
    "lambda1", "lambda2", "fov", "render_preview", "ready", "tile_histogram", "device",
};

inline int packet_id(const std::string& name) {
  for (size_t i = 0; i < kPacketTypes.size(); ++i)
    if (kPacketTypes[i] == name) return (int)i;
  return -1;
}

// AsyncTask (AsyncTask.hpp:22-66): run one function on a thread; wait for it.
class AsyncTask {
 public:
  void run(std::function<void()> f) {
    waitForCompletion();
    running_ = true;
    t_ = std::thread([this, f] {
      f();
      running_ = false;
    });
  }
  void waitForCompletion() {
    if (t_.joinable()) t_.join();
  }
  bool isRunning() const { return running_; }
  ~AsyncTask() { waitForCompletion(); }

 private:
  std::thread t_;
  std::atomic<bool> running_{false};
};

class InterfaceServer {
 public:
  // InterfaceServer.hpp:230-244 (defaults kept)
  struct State {
    float envRotationDegrees = 0.f;
    float envRotationDegrees2 = 0.f;
    float exposure = 0.f;
    float gamma = 2.2f;
    float X = 640.f;
    float Y = 360.f;
    float Z = 1.f;
    float lambda1 = 1.f;
    float lambda2 = 1.f;
    float fov = 90.f;
    std::string device = "cpu";
    bool stop = false;
    bool detach = false;
  };

  // bind_host: the address to listen on (an IPv4 literal); the default is
  // loopback -- a render server is reachable from other hosts only when the
  // caller names an address (bin/splat --ui-host)
  explicit InterfaceServer(int port, const char* bind_host = "127.0.0.1") : port_(port), host_(bind_host) {}
  ~InterfaceServer() { stop(); }

  // Launch the server thread and block until a client is connected and the
  // "ready" exchange is done (InterfaceServer.hpp:272-278).  The initial state
  // (e.g. the render server's fov and device) is seeded first.
  bool start(const State& initial) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      state_ = initial;
    }
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (listen_fd_ < 0) return false;
    int one = 1;
    ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    if (::inet_pton(AF_INET, host_.c_str(), &addr.sin_addr) != 1) return false;
    addr.sin_port = htons((uint16_t)port_);
    if (::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) != 0 || ::listen(listen_fd_, 1) != 0) return false;
    std::printf("[info] User interface server listening on port %d\n", port_);
    std::fflush(stdout);
    conn_ = ::accept(listen_fd_, nullptr, nullptr);
    if (conn_ < 0) return false;
    ::setsockopt(conn_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::printf("[info] User interface client connected.\n");
    // syncWithClient(sender, receiver, "ready")
    send_packet("ready", nullptr, 0);
    uint32_t type = 0;
    std::vector<uint8_t> payload;
    do {
      if (!recv_packet(type, payload)) return false;
    } while (type != (uint32_t)packet_id("ready"));
    thread_ = std::thread([this] { communicate(); });
    return true;
  }

  void stop() {
    stop_server_ = true;
    if (thread_.joinable()) thread_.join();
    if (conn_ >= 0) ::close(conn_);
    if (listen_fd_ >= 0) ::close(listen_fd_);
    conn_ = listen_fd_ = -1;
  }

  // Return a copy of the state and mark it consumed (InterfaceServer.hpp:247-251).
  State consumeState() {
    std::lock_guard<std::mutex> lk(mu_);
    updated_ = false;
    return state_;
  }
  bool stateChanged() const { return updated_; }

  void updateFov(float fovRadians) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      state_.fov = fovRadians;
    }
    send_packet("fov", &fovRadians, 4);
  }

  void sendHistogram(const std::vector<uint32_t>& data) {
    std::vector<uint8_t> p(8 + data.size() * 4);
    const uint64_t n = data.size();
    std::memcpy(p.data(), &n, 8);
    if (n) std::memcpy(p.data() + 8, data.data(), data.size() * 4);
    send_packet("tile_histogram", p.data(), p.size());
  }

  // A BGR24 frame, zlib-compressed (no FFmpeg in this build).
  bool sendPreviewImage(const uint8_t* bgr, int width, int height) {
    const uLong raw = (uLong)width * height * 3;
    uLongf zlen = compressBound(raw);
    std::vector<uint8_t> p(12 + zlen);
    const int32_t w = width, h = height;
    const uint32_t codec = 1;
    std::memcpy(p.data(), &w, 4);
    std::memcpy(p.data() + 4, &h, 4);
    std::memcpy(p.data() + 8, &codec, 4);
    if (compress2(p.data() + 12, &zlen, bgr, raw, 1) != Z_OK) return false;
    p.resize(12 + zlen);
    return send_packet("render_preview", p.data(), p.size());
  }

  bool connected() const { return !disconnected_; }

 private:
  void communicate() {
    uint32_t type = 0;
    std::vector<uint8_t> p;
    while (!stop_server_) {
      pollfd pf{conn_, POLLIN, 0};
      const int pr = ::poll(&pf, 1, 5);
      if (pr < 0) break;
      if (pr == 0) continue;
      if (!recv_packet(type, p)) break;
      apply(type, p);
    }
    if (!stop_server_) {  // the client went away: stop the render loop
      std::lock_guard<std::mutex> lk(mu_);
      disconnected_ = true;
      state_.stop = true;
      updated_ = true;
    }
    std::printf("[info] User interface server Tx/Rx loop exited.\n");
    std::fflush(stdout);
  }

  void apply(uint32_t type, const std::vector<uint8_t>& p) {
    if (type >= kPacketTypes.size()) return;
    const std::string& name = kPacketTypes[type];
    std::lock_guard<std::mutex> lk(mu_);
    auto f32 = [&](float& dst) {
      if (p.size() >= 4) std::memcpy(&dst, p.data(), 4);
    };
    if (name == "env_rotation") f32(state_.envRotationDegrees);
    else if (name == "env_rotation_2") f32(state_.envRotationDegrees2);
    else if (name == "exposure") f32(state_.exposure);
    else if (name == "gamma") f32(state_.gamma);
    else if (name == "X") f32(state_.X);
    else if (name == "Y") f32(state_.Y);
    else if (name == "Z") f32(state_.Z);
    else if (name == "lambda1") f32(state_.lambda1);
    else if (name == "lambda2") f32(state_.lambda2);
    else if (name == "fov") {
      float deg = 0.f;
      f32(deg);
      state_.fov = (float)((double)deg * (M_PI / 180.f));  // to radians (InterfaceServer.hpp:191-193)
    } else if (name == "stop") {
      state_.stop = !p.empty() && p[0] != 0;
    } else if (name == "detach") {
      state_.detach = !p.empty() && p[0] != 0;
    } else if (name == "device") {
      // u64 length + bytes; a length the payload does not hold (or an
      // implausible one) is ignored, never trusted
      if (p.size() < 8) return;
      uint64_t n = 0;
      std::memcpy(&n, p.data(), 8);
      if (n > p.size() - 8 || n > kMaxDeviceName) return;
      state_.device.assign((const char*)p.data() + 8, (size_t)n);
    } else {
      return;  // not a client -> server packet
    }
    updated_ = true;
  }

  bool send_all(const void* d, size_t n) {
    const char* c = (const char*)d;
    while (n) {
      const ssize_t k = ::send(conn_, c, n, MSG_NOSIGNAL);
      if (k <= 0) return false;
      c += k;
      n -= (size_t)k;
    }
    return true;
  }

  bool recv_all(void* d, size_t n) {
    char* c = (char*)d;
    while (n) {
      const ssize_t k = ::recv(conn_, c, n, 0);
      if (k <= 0) return false;
      c += k;
      n -= (size_t)k;
    }
    return true;
  }

  bool send_packet(const char* name, const void* payload, size_t n) {
    std::lock_guard<std::mutex> lk(send_mu_);
    if (conn_ < 0 || disconnected_) return false;
    const uint32_t hdr[2] = {(uint32_t)packet_id(name), (uint32_t)n};
    return send_all(hdr, 8) && (n == 0 || send_all(payload, n));
  }

  bool recv_packet(uint32_t& type, std::vector<uint8_t>& payload) {
    uint32_t hdr[2];
    if (!recv_all(hdr, 8)) return false;
    if (hdr[1] > (64u << 20)) return false;
    type = hdr[0];
    payload.resize(hdr[1]);
    return hdr[1] == 0 || recv_all(payload.data(), hdr[1]);
  }

  static constexpr uint64_t kMaxDeviceName = 64;
  int port_;
  std::string host_;
  int listen_fd_ = -1, conn_ = -1;
  std::thread thread_;
  std::atomic<bool> stop_server_{false};
  std::atomic<bool> updated_{false};
  std::atomic<bool> disconnected_{false};
  std::mutex mu_, send_mu_;
  State state_;
};

}  // namespace gsui
