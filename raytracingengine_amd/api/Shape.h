// Shape.h — drop-in name for the reference header; provides Transform, Material, HitType, HitInfo, Sphere, Plane, Triangle, Model (reference Shape.h).
#pragma once
#include "rtamd/shapes.hpp"
