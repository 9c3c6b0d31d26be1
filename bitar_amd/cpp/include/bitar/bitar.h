// bitar/bitar.h -- umbrella header of the MI355X bitar front-end.
#pragma once

#include "bitar/arrow_codec.h"
#include "bitar/config.h"
#include "bitar/device.h"
#include "bitar/driver.h"
#include "bitar/hip_device.h"
#include "bitar/memory_pool.h"
#include "bitar/type_fwd.h"
#include "bitar/util.h"
