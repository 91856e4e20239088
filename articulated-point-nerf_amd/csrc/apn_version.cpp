// Library identification string (apn_version in include/apn_hip.h).
#include "../../include/apn_hip.h"
#ifdef APN_DEBUG_BUILD
extern "C" const char* apn_version(void) { return "apn_hip 0.1 gfx950 debug"; }
#else
extern "C" const char* apn_version(void) { return "apn_hip 0.1 gfx950"; }
#endif
