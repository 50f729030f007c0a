// n_links = 7: every kernel family of this link count (fgx_ep_nl.h).
#define FGX_NL 7
#include "fgx_ep_nl.h"
