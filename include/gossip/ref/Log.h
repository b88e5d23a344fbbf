// include/gossip/ref/Log.h -- forwarding header: the reference's Log.h on the MI355X engine.
//
// A driver written against /root/reference compiles unchanged against this directory in place
// of the reference's own headers (put it first on the include path): Log (Log.h:28-40)
// come from the C++ facade over libgossip_amd.so (../mp1_facade.hpp), with rand() / srand() on
// the engine's draw stream (gsp_rand_interpose.h).  INTEGRATION.md section 1 shows the build.
#include "gsp_rand_interpose.h"
