// Umbrella header of the MI355X-native xerus hot path (reference include/xerus.h:31-64).
#pragma once
#include "xerus/basic.h"
#include "xerus/index.h"
#include "xerus/indexedTensor.h"
#include "xerus/indexedTensor_tensor_factorisations.h"
#include "xerus/misc/fileIO.h"
#include "xerus/misc/random.h"
#include "xerus/tensor.h"
#include "xerus/tensorNetwork.h"
#include "xerus/ttNetwork.h"
#include "xerus/algorithms/als.h"
#include "xerus/measurments.h"
#include "xerus/algorithms/adf.h"

namespace xerus {
namespace gpu {
/// device of the calling thread's context (default 0, or $XERUS_DEVICE); must be set before first use
void set_device(int _device);
int device();
/// the calling thread's xerus_amd handle (stream + caching allocator)
struct xrs_handle_s* handle();
void synchronize();
}  // namespace gpu
}  // namespace xerus
