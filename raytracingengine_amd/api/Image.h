// Image.h — drop-in name for the reference header; provides writePPM (reference Image.h) + device tonemap.
#pragma once
#include "rtamd/image.hpp"
