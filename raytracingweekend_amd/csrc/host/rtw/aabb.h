#pragma once
#include "ray.h"  // aabb lives next to ray in this API
