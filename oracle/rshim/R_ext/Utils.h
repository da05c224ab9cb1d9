/* oracle/rshim/R_ext/Utils.h — nothing beyond R.h is needed. */
#include "../R.h"
