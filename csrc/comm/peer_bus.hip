// Peer data plane regions (see peer_bus.h).
#include "peer_bus.h"

#include <vector>

#include <cstring>
#include <stdexcept>

namespace psx {
namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("PeerBus: ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

PeerRegion::PeerRegion(const PeerLayout& lay, int device) : lay_(lay) {
  if (lay.P < 1 || lay.NS < 1 || lay.slots < 1) throw std::invalid_argument("PeerRegion: empty layout");
  ck(hipSetDevice(device), "hipSetDevice");
  // fine-grained: another GPU's system-scope stores / loads over xGMI are coherent
  // with this GPU's (tools/peer_probe.hip: exported, mapped and ping-ponged)
  ck(hipExtMallocWithFlags(&p_, lay.bytes(), hipDeviceMallocFinegrained), "hipExtMallocWithFlags(fine-grained)");
  ck(hipMemset(p_, 0, lay.bytes()), "hipMemset");
  ck(hipDeviceSynchronize(), "sync");
}

PeerRegion::~PeerRegion() {
  if (p_) (void)hipFree(p_);
}

void PeerRegion::fill_tags(unsigned value) {
  std::vector<unsigned> h((size_t)lay_.slots * lay_.NS, value);
  ck(hipMemcpy(static_cast<char*>(p_) + lay_.tag_off(), h.data(), h.size() * 4, hipMemcpyHostToDevice), "tags");
  ck(hipDeviceSynchronize(), "sync");
}

std::string PeerRegion::handle() const {
  hipIpcMemHandle_t h;
  ck(hipIpcGetMemHandle(&h, p_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

PeerMapping::PeerMapping(const std::string& handle, const PeerLayout& lay) : lay_(lay) {
  if (handle.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("PeerMapping: bad handle");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.data(), sizeof(h));
  ck(hipIpcOpenMemHandle(&p_, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
}

PeerMapping::~PeerMapping() { close(); }

void PeerMapping::close() {
  if (p_) (void)hipIpcCloseMemHandle(p_);
  p_ = nullptr;
}

}  // namespace psx
