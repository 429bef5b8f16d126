/* abi_check.c — the C-ABI is plain C: this file is compiled with gcc -std=c99
 * -pedantic against include/tips_hip.h and linked against libtips_hip.so
 * (tests/test_abi.py::test_header_is_c99). It calls only entry points that
 * need no GPU, the way a cgo/JNI/ctypes binding would. */
#include <stdio.h>
#include <string.h>

#include "tips_hip.h"

int main(void) {
  int64_t b = -1, e = -1;
  int64_t table[2 * TIPS_REQUEST_WORDS];
  if (tips_is_initialize() || tips_size() != -1 || tips_rank() != -1) return 1;
  if (tips_unique_id_bytes() != 128) return 2;
  if (tips_chunk_bounds(4099, 4, TIPS_FLOAT32, 3, &b, &e) != TIPS_OK || b != 3264 || e != 4099) return 3;
  if (tips_allreduce(NULL, NULL, 8, TIPS_FLOAT32, TIPS_OP_SUM, NULL) != TIPS_ERR_NOT_INITIALIZED) return 4;
  if (strstr(tips_last_error(), "tips_init") == NULL) return 5;
  if (tips_allreduce(NULL, NULL, 8, TIPS_FLOAT32, TIPS_OP_MIN, NULL) != TIPS_ERR_UNSUPPORTED) return 6;
  memset(table, 0, sizeof table);
  table[0] = TIPS_REQ_ALLREDUCE;
  table[1] = TIPS_FLOAT32;
  table[2] = 1;
  table[3] = 10;
  memcpy(table + TIPS_REQUEST_WORDS, table, TIPS_REQUEST_WORDS * sizeof(int64_t));
  if (tips_check_requests(table, 2) != TIPS_OK) return 7;
  table[TIPS_REQUEST_WORDS + 1] = TIPS_FLOAT64;
  if (tips_check_requests(table, 2) != TIPS_ERR_MISMATCH) return 8;
  printf("%s | %s\n", tips_version(), tips_last_error());
  return 0;
}
