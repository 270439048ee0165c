// Flat batches planned on the device (placeholder until the device planner lands).
#include "engine_core.hpp"

namespace hcphmm {
namespace eng {

int plan_flat_device(Device&, const Src&, const PartSpec&, Slot*, bool, Part** out)
{
    *out = nullptr;
    return HC_PHMM_OK;
}

}  // namespace eng
}  // namespace hcphmm
