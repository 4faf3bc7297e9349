// VMAS contact-physics envs (DGPPO_ENGINE_VMAS_WHEEL / _TRANSPORT): entry points called from the
// dgppo_env_* C-ABI in env_step.hip when cfg->engine names a VMAS env.  Defined in vmas.hip.
#pragma once
#include "dgppo_hip.h"

namespace dgppo {
namespace vmas {

bool is_vmas(const dgppo_env_cfg* c);
int finalize(dgppo_env_cfg* c);
int validate(const dgppo_env_cfg* c);
int step(const dgppo_env_cfg* c, const dgppo_env_step_io* io, void* stream);
int reset(const dgppo_env_cfg* c, const dgppo_env_reset_io* io, void* stream);
int rollout(const dgppo_env_cfg* c, const dgppo_env_rollout_io* r, void* stream);

}  // namespace vmas
}  // namespace dgppo
