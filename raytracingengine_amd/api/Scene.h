// Scene.h — drop-in name for the reference header; provides Scene (reference Scene.h), rendered on the MI355X.
#pragma once
#include "rtamd/scene.hpp"
