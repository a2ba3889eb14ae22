// rt_packet_area.hip — the packet kernel's area-light variants (rt_packet.hip), compiled in their
// own translation unit with the compiler's default scheduling strategy.
#define RT_PACKET_AREA_TU 1
#include "rt_packet.hip"
