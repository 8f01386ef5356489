/* placeholder: H.264 oracle under construction */
#include "oracle.h"
int oracle_h264_decode(const uint8_t *data, long size, int flags, OraclePicture *pic){return -1;}
