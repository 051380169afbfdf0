// Peer-to-peer exchange buffers (see p2p.h).
#include "p2p.h"

#include <cstring>
#include <stdexcept>

namespace sml {

#define P2P_CHECK(expr)                                                                         \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess) throw std::runtime_error(std::string("P2PExchange: ") + #expr + ": " + \
                                                   hipGetErrorString(_e));                      \
  } while (0)

namespace {
constexpr uint64_t kMagic = 0x534d4c5032500000ull;   // "SMLP2P" + rank in the low bits
}

void P2PExchange::alloc_buffer(int r) {
  void* p = nullptr;
  const size_t bytes = buffer_bytes();
  P2P_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
  P2P_CHECK(hipMemset(p, 0, bytes));
  const uint64_t magic = kMagic | (uint64_t)r;
  P2P_CHECK(hipMemcpy(static_cast<char*>(p) + bytes - 64, &magic, 8, hipMemcpyHostToDevice));
  own_.push_back(p);
}

P2PExchange::P2PExchange(int device, int rank, int world, int64_t slots)
    : device_(device), rank_(rank), world_(world), slots_(slots) {
  if (world < 1 || rank < 0 || rank >= world || slots < 1 || slots > (1 << 24))
    throw std::invalid_argument("P2PExchange: bad rank / world / slots");
  P2P_CHECK(hipSetDevice(device_));
  alloc_buffer(rank_);
  P2P_CHECK(hipMalloc(&status_, sizeof(int)));
  P2P_CHECK(hipMemset(status_, 0, sizeof(int)));
}

P2PExchange* P2PExchange::local(int device, int world, int64_t slots) {
  if (world < 1 || slots < 1 || slots > (1 << 24)) throw std::invalid_argument("P2PExchange: bad world / slots");
  auto* x = new P2PExchange();
  x->device_ = device;
  x->rank_ = 0;
  x->world_ = world;
  x->slots_ = slots;
  P2P_CHECK(hipSetDevice(device));
  for (int r = 0; r < world; ++r) x->alloc_buffer(r);
  x->peers_ = x->own_;
  P2P_CHECK(hipMalloc(&x->status_, sizeof(int)));
  P2P_CHECK(hipMemset(x->status_, 0, sizeof(int)));
  x->publish_peers();
  return x;
}

P2PExchange::~P2PExchange() {
  if (hipSetDevice(device_) != hipSuccess) return;
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  for (void* p : own_) hipFree(p);
  if (peers_dev_) hipFree(peers_dev_);
  if (status_) hipFree(status_);
}

std::string P2PExchange::handle() const {
  hipIpcMemHandle_t h;
  P2P_CHECK(hipSetDevice(device_));
  P2P_CHECK(hipIpcGetMemHandle(&h, own_.at(0)));
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void P2PExchange::open(const std::vector<std::string>& handles) {
  if ((int)handles.size() != world_) throw std::invalid_argument("P2PExchange: need one handle per rank");
  if (peers_dev_) throw std::logic_error("P2PExchange: already open");
  P2P_CHECK(hipSetDevice(device_));
  peers_.assign((size_t)world_, nullptr);
  peers_[(size_t)rank_] = own_.at(0);
  const size_t bytes = buffer_bytes();
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    if (handles[(size_t)r].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("P2PExchange: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[(size_t)r].data(), sizeof(h));
    void* p = nullptr;
    P2P_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
    opened_.push_back(p);
    peers_[(size_t)r] = p;
    // validate the mapping by DMA before any kernel dereferences it: the peer's magic word
    uint64_t magic = 0;
    P2P_CHECK(hipMemcpy(&magic, static_cast<char*>(p) + bytes - 64, 8, hipMemcpyDeviceToHost));
    if (magic != (kMagic | (uint64_t)r))
      throw std::runtime_error("P2PExchange: peer " + std::to_string(r) + " buffer failed validation");
  }
  publish_peers();
}

void P2PExchange::publish_peers() {
  std::vector<uint64_t*> v(peers_.size());
  for (size_t i = 0; i < peers_.size(); ++i) v[i] = static_cast<uint64_t*>(peers_[i]);
  P2P_CHECK(hipMalloc(&peers_dev_, v.size() * sizeof(uint64_t*)));
  P2P_CHECK(hipMemcpy(peers_dev_, v.data(), v.size() * sizeof(uint64_t*), hipMemcpyHostToDevice));
}

int P2PExchange::status() const {
  int s = 0;
  P2P_CHECK(hipSetDevice(device_));
  P2P_CHECK(hipMemcpy(&s, status_, sizeof(int), hipMemcpyDeviceToHost));
  return s;
}

void P2PExchange::clear() {
  P2P_CHECK(hipSetDevice(device_));
  const size_t bytes = buffer_bytes();
  for (size_t i = 0; i < own_.size(); ++i) {
    P2P_CHECK(hipMemset(own_[i], 0, bytes - 64));
  }
  P2P_CHECK(hipDeviceSynchronize());
}

void P2PExchange::reset_status() {
  P2P_CHECK(hipSetDevice(device_));
  P2P_CHECK(hipMemset(status_, 0, sizeof(int)));
}

}  // namespace sml
