// Forced-include prelude used ONLY when compiling the reference's own sources
// (/root/reference/cpp/{core,game}) into oracle/_ref/refgen.  It works around
// the reference's compile blockers without editing or copying its files:
//  - core/global.h:343-346 uses unqualified `string`
//  - game/board.h:24 uses Spot/Player/Direction before their typedefs (B1)
// The remaining blockers are patched by line-addressed sed in build_ref.sh.
#include <string>
#include <vector>
#include <cstdint>
using std::string;
using std::vector;
typedef short Spot;
typedef int8_t Player;
typedef int8_t Direction;
