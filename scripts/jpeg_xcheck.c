/* Development cross-check (not product, not oracle): decode a JPEG with the
 * system's IJG libjpeg 9 (where one is installed, e.g. /opt/conda) exactly as
 * OpenCV 3.4's JpegDecoder drives it -- default parameters, JCS_RGB out --
 * and write BGR bytes, so tests can compare oracle/cg_oracle_jpeg.c with it.
 *   gcc -I<inc> jpeg_xcheck.c -o jpeg_xcheck <libjpeg.so.9>
 *   jpeg_xcheck IN.jpg OUT.bgr */
#include <stdio.h>
#include <stdlib.h>

#include <jpeglib.h>

int main(int argc, char **argv)
{
    if (argc != 3) return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    struct jpeg_decompress_struct c;
    struct jpeg_error_mgr e;
    c.err = jpeg_std_error(&e);
    jpeg_create_decompress(&c);
    jpeg_stdio_src(&c, f);
    jpeg_read_header(&c, TRUE);
    if (c.num_components == 3) c.out_color_space = JCS_RGB;
    jpeg_start_decompress(&c);
    int w = (int)c.output_width, h = (int)c.output_height, n = c.output_components;
    unsigned char *buf = malloc((size_t)w * h * n);
    while (c.output_scanline < c.output_height) {
        unsigned char *row = buf + (size_t)c.output_scanline * w * n;
        jpeg_read_scanlines(&c, &row, 1);
    }
    jpeg_finish_decompress(&c);
    jpeg_destroy_decompress(&c);
    fclose(f);
    FILE *o = fopen(argv[2], "wb");
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        if (n == 3) { unsigned char p[3] = {buf[3 * i + 2], buf[3 * i + 1], buf[3 * i]}; fwrite(p, 1, 3, o); }
        else fwrite(buf + i, 1, 1, o);
    }
    fclose(o);
    free(buf);
    return 0;
}
