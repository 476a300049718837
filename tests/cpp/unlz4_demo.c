/* unlz4_demo.c -- the reference decoder's command-line pattern (smallz4cat.c:60-106, 373-417)
 * on include/smallz4cat_amd.h: a file or stdin in, stdout out, optional -D dictionary.
 * Used by tests/test_abi.py (compiles) and tests/test_unlz4.py (runs). */
#include <stdio.h>

#include "smallz4cat_amd.h"

struct UserPtr {
  FILE* in;
  FILE* out;
  unsigned char buf[4096];
  unsigned int pos, available;
};

static unsigned char getByteFromIn(void* userPtr)
{
  struct UserPtr* u = (struct UserPtr*)userPtr;
  if (u->pos == u->available) {
    u->pos = 0;
    u->available = (unsigned int)fread(u->buf, 1, sizeof u->buf, u->in);
    if (u->available == 0) sz4cat_error("out of data");
  }
  return u->buf[u->pos++];
}

static void sendBytesToOut(const unsigned char* data, unsigned int numBytes, void* userPtr)
{
  struct UserPtr* u = (struct UserPtr*)userPtr;
  if (data != NULL && numBytes > 0) fwrite(data, 1, numBytes, u->out);
}

int main(int argc, const char* argv[])
{
  struct UserPtr user;
  const char* dictionary = NULL;
  int i;
  user.in = stdin;
  user.out = stdout;
  user.pos = user.available = 0;
  for (i = 1; i < argc; i++) {
    if (argv[i][0] == '-' && argv[i][1] == 'D') {
      if (i + 1 >= argc) sz4cat_error("no dictionary filename found");
      dictionary = argv[++i];
      continue;
    }
    if (argv[i][0] != '-' || argv[i][1] != '\0') {
      user.in = fopen(argv[i], "rb");
      if (!user.in) sz4cat_error("file not found");
    }
  }
  unlz4_userPtr(getByteFromIn, sendBytesToOut, dictionary, &user);
  return 0;
}
