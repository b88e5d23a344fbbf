// include/gossip/ref/gsp_rand_interpose.h -- rand() / srand() onto the engine's draw stream.
//
// The reference's Application seeds libc with srand(time(NULL)) (Application.cpp:50, 96) and
// draws rand() in fail() (Application.cpp:182, 189) from the stream EmulNet::ENsend draws from
// (EmulNet.cpp:89).  The engine owns that stream, so in a translation unit that includes the
// forwarding headers of this directory, rand() and srand() are the facade's gsp_mp1_rand() /
// gsp_mp1_srand() (mp1_facade.hpp).  Function-like macros, defined after the standard headers
// the facade includes: `std::rand` and `using ::rand` in later headers are untouched, and no
// other object of the program (libraries included) sees a different rand().
#ifndef GOSSIP_REF_GSP_RAND_INTERPOSE_H
#define GOSSIP_REF_GSP_RAND_INTERPOSE_H
#include "../mp1_facade.hpp"
#define srand(seed) gsp_mp1_srand(seed)
#define rand() gsp_mp1_rand()
#endif
