/* EarthBuiltin's texels, linked into libshirley_host.so the way the reference links its JPEG with
 * include_bytes! (image_texture.rs:11,18-20): no run-time file lookup, so every copy of the library
 * (lib/, lib/diag/, exp/<variant>/) renders the earth scene without SHIRLEY_ASSETS.
 * The payload is assets/earthmap.rgb8.gz (the JPEG decoded once by tools/decode_earthmap.py);
 * the Makefile passes the assets directory with -Wa,-I so .incbin finds it. */
        .section .rodata
        .balign 16
        .globl  shirley_earth_rgb8_gz
        .hidden shirley_earth_rgb8_gz
        .type   shirley_earth_rgb8_gz, @object
shirley_earth_rgb8_gz:
        .incbin "earthmap.rgb8.gz"
        .globl  shirley_earth_rgb8_gz_end
        .hidden shirley_earth_rgb8_gz_end
shirley_earth_rgb8_gz_end:
        .byte 0
        .section .note.GNU-stack,"",@progbits
