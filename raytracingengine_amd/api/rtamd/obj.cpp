// rtamd/obj.cpp — see obj.hpp.
#include "rtamd/obj.hpp"

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <vector>

namespace rtamd {

namespace {

// A real as tinyobjloader v1.0.x reads it (tryParseDouble, tiny_obj_loader.h:447-587 of the
// copy vendored by the reference): [sign] digits ["." digits] [("e"|"E") [sign] digits], the
// integer digits accumulated as mantissa*10 + d, fraction digit k added as d*10^-k (a table of
// double literals for k < 8, pow(10, -k) beyond), the result ldexp(mantissa*5^e, e); anything
// that does not start with a sign or a digit, or an empty exponent, reads as `fallback`.  Not
// correctly rounded (".5" reads as 0, some long fractions differ from strtod in the last bit),
// which is why it is restated instead of calling strtod.
double tinyobj_real(const std::string& s, double fallback) {
    static const double kPow[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
    size_t i = 0;
    const size_t n = s.size();
    if (n == 0) return fallback;
    char sign = '+';
    if (s[i] == '+' || s[i] == '-') sign = s[i++];
    else if (!std::isdigit(static_cast<unsigned char>(s[i]))) return fallback;
    double mantissa = 0.0;
    int digits = 0;
    while (i < n && std::isdigit(static_cast<unsigned char>(s[i]))) {
        mantissa *= 10;
        mantissa += static_cast<int>(s[i] - '0');
        ++i;
        ++digits;
    }
    if (digits == 0) return fallback;
    int exponent = 0;
    if (i < n && s[i] == '.') {
        ++i;
        for (int k = 1; i < n && std::isdigit(static_cast<unsigned char>(s[i])); ++k, ++i)
            mantissa += static_cast<int>(s[i] - '0') * (k < 8 ? kPow[k] : std::pow(10.0, -k));
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        ++i;
        char esign = '+';
        if (i < n && (s[i] == '+' || s[i] == '-')) esign = s[i++];
        else if (!(i < n && std::isdigit(static_cast<unsigned char>(s[i])))) return fallback;
        int ed = 0;
        while (i < n && std::isdigit(static_cast<unsigned char>(s[i]))) {
            exponent = exponent * 10 + static_cast<int>(s[i] - '0');
            ++i;
            ++ed;
        }
        if (ed == 0) return fallback;
        if (esign == '-') exponent = -exponent;
    }
    return (sign == '+' ? 1 : -1) *
           (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
}

// One face corner "i", "i/t", "i//n" or "i/t/n" -> 0-based position index, as tinyobj reads
// it: the leading integer (atoi), 1-based, 0 taken as 0, negative relative to the vertices read
// so far.
long corner_index(const std::string& tok, long nverts) {
    const long i = std::atoi(tok.c_str());
    if (i > 0) return i - 1;
    if (i == 0) return 0;
    return nverts + i;
}

}  // namespace

Model LoadObject(const std::string& modelName, const Transform& transform,
                 const Material& material) {
    std::ifstream in(modelName);
    if (!in) {
        std::cerr << "OBJ ERR: Cannot open file [" << modelName << "]" << std::endl;
        throw std::runtime_error("Failed to load/parse .obj.");
    }
    std::vector<Vec3> positions;
    std::vector<int> indices;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string kw;
        if (!(ls >> kw)) continue;
        if (kw == "v") {
            std::string sx, sy, sz;
            ls >> sx >> sy >> sz;
            const float x = static_cast<float>(tinyobj_real(sx, 0.0));
            const float y = static_cast<float>(tinyobj_real(sy, 0.0));
            const float z = static_cast<float>(tinyobj_real(sz, 0.0));
            positions.emplace_back(static_cast<double>(x), static_cast<double>(y),
                                   static_cast<double>(z));
        } else if (kw == "f") {
            std::vector<long> face;
            std::string tok;
            while (ls >> tok) {
                const long i = corner_index(tok, static_cast<long>(positions.size()));
                if (i < 0 || i >= static_cast<long>(positions.size()))
                    throw std::runtime_error("OBJ face index out of range in " + modelName);
                face.push_back(i);
            }
            if (face.size() < 3) continue;
            for (size_t k = 2; k < face.size(); ++k) {  // fan from the first corner
                indices.push_back(static_cast<int>(face[0]));
                indices.push_back(static_cast<int>(face[k - 1]));
                indices.push_back(static_cast<int>(face[k]));
            }
        }
    }
    return Model(indices, transform, material, positions);
}

}  // namespace rtamd
