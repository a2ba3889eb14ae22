// Light.h — drop-in name for the reference header; provides Light (reference Light.h).
#pragma once
#include "rtamd/light.hpp"
