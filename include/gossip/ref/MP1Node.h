// include/gossip/ref/MP1Node.h -- forwarding header: the reference's MP1Node.h on the MI355X engine.
//
// A driver written against /root/reference compiles unchanged against this directory in place
// of the reference's own headers (put it first on the include path): MP1Node, MessageHdr, MsgTypes, TREMOVE / TFAIL (MP1Node.h:21-86)
// come from the C++ facade over libgossip_amd.so (../mp1_facade.hpp), with rand() / srand() on
// the engine's draw stream (gsp_rand_interpose.h).  INTEGRATION.md section 1 shows the build.
#include "gsp_rand_interpose.h"
