// Model families whose native graphs are not wired yet fail loudly at creation.
#include "sa/engine.h"

namespace sa {
#ifndef SA_HAVE_HITNET
std::unique_ptr<StereoEngine> make_hitnet(const EngineConfig& cfg) {
  throw Error("HITNet native engine not built (preset " + cfg.model + ")");
}
#endif
}  // namespace sa
