// Math.h — drop-in name for the reference header; provides Vec3, Color, Rayon, Camera (reference Math.h).
#pragma once
#include "rtamd/math.hpp"
