/*
 * smallpt_gl.c -- the optional display: smallpt's host loop in an X11 window,
 * each frame handed to OpenGL through HIP-GL interop (bdpt_gl_register_pbo / bdpt_gl_publish,
 * include/bdpt.h) instead of a read-back through the host.
 *
 *   smallpt_gl [<width> <height> <scene.scn>] [--device D] [--batch B] [--frames N] [--dat PATH]
 *
 * The reference's display path, without GLUT (not in this image -- Xlib + GLX instead):
 *   InitGlut / ReshapeFunc (display_func.c:439-470, :257-270) -> X window, GLX context, orthographic
 *       projection on the unit square
 *   CreatePBO + cudaGLRegisterBufferObject (smallpt_cpu.c:112-123) -> a GL_PIXEL_UNPACK_BUFFER of
 *       4*W*H bytes registered with bdpt_gl_register_pbo; createTexture (:125-140) -> RGBA8 texture
 *   IdleFunc (display_func.c:192-217) -> the first frame is the light pass + one path pass
 *       (UpdateRendering2 then UpdateRendering), every later frame B path passes (B = 1 is the
 *       reference's one pass per idle call), then bdpt_gl_publish (map, pixels, unmap)
 *   DisplayFunc (:219-255) -> the PBO into the texture (glTexSubImage2D from offset 0), a textured
 *       quad, the help panel when toggled on (text from an X core font via glXUseXFont: GLUT's
 *       bitmap fonts are not available), buffer swap
 *   KeyFunc / SpecialFunc (:278-437) -> the same keys: Escape quits, h toggles help, i prints the
 *       camera, the others go through smallpt_app.h's key() (camera / scene edits, p = SavePPM)
 * --frames N stops after N displayed frames (0 = until Escape or the window is closed).
 * Exit status 2 when no X display can be opened (the GPU nodes are headless).
 */
#define GL_GLEXT_PROTOTYPES 1
#include <GL/gl.h>
#include <GL/glext.h>
#include <GL/glx.h>
#include <X11/Xlib.h>
#include <X11/Xutil.h>
#include <X11/keysym.h>

#include "smallpt_app.h"

typedef struct {
    Display *dpy;
    Window win;
    GLXContext glc;
    GLuint pbo, tex, font;
    int print_help;
} view;

static const char *const help_lines[] = {
    "h - toggle Help",
    "arrow Keys - rotate camera left/right/up/down",
    "a and d - move camera left and right",
    "w and s - move camera forward and backward",
    "r and f - move camera up and down",
    "PageUp and PageDown - move camera target up and down",
    "+ and - - to select next/previous object",
    "2, 3, 4, 5, 6, 8, 9 - to move selected object",
};

static void print_string(const view *v, const char *s)
{
    if (!v->font) return;
    glListBase(v->font - 32);
    glCallLists((GLsizei)strlen(s), GL_UNSIGNED_BYTE, s);
}

/* ReshapeFunc display_func.c:257-270 */
static void reshape(int w, int hgt)
{
    glViewport(0, 0, w, hgt);
    glClearColor(0.0, 0.0, 0.0, 1.0);
    glDisable(GL_DEPTH_TEST);
    glMatrixMode(GL_MODELVIEW);
    glLoadIdentity();
    glMatrixMode(GL_PROJECTION);
    glLoadIdentity();
    glOrtho(0.0, 1.0, 0.0, 1.0, 0.0, 1.0);
}

/* DisplayFunc display_func.c:219-255 */
static void display(const view *v, const host *h)
{
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, v->pbo);
    glClear(GL_COLOR_BUFFER_BIT);
    glBindTexture(GL_TEXTURE_2D, v->tex);
    glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, h->width, h->height, GL_RGBA, GL_UNSIGNED_BYTE, NULL);
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
    glEnable(GL_TEXTURE_2D);
    glBegin(GL_QUADS);
    glTexCoord2f(0.0f, 0.0f); glVertex3f(0.0f, 0.0f, 0.0f);
    glTexCoord2f(0.0f, 1.0f); glVertex3f(0.0f, 1.0f, 0.0f);
    glTexCoord2f(1.0f, 1.0f); glVertex3f(1.0f, 1.0f, 0.0f);
    glTexCoord2f(1.0f, 0.0f); glVertex3f(1.0f, 0.0f, 0.0f);
    glEnd();
    glDisable(GL_TEXTURE_2D);
    if (v->print_help) {                         /* PrintHelp display_func.c:82-110 */
        glPushMatrix();
        glLoadIdentity();
        glOrtho(-0.5, 639.5, -0.5, 479.5, -1.0, 1.0);
        glEnable(GL_BLEND);
        glBlendFunc(GL_SRC_ALPHA, GL_ONE_MINUS_SRC_ALPHA);
        glColor4f(0.f, 0.f, 0.5f, 0.5f);
        glRecti(40, 40, 600, 440);
        glColor3f(1.f, 1.f, 1.f);
        glRasterPos2i(300, 420);
        print_string(v, "Help");
        for (int k = 0; k < (int)(sizeof help_lines / sizeof help_lines[0]); k++) {
            glRasterPos2i(60, 390 - 30 * k);
            print_string(v, help_lines[k]);
        }
        glDisable(GL_BLEND);
        glPopMatrix();
    }
    glFlush();
    glXSwapBuffers(v->dpy, v->win);
}

/* KeyFunc / SpecialFunc display_func.c:278-437; returns 0 to quit */
static int on_key(view *v, host *h, XKeyEvent *e)
{
    char buf[8];
    KeySym ks;
    const int n = XLookupString(e, buf, (int)sizeof buf, &ks, NULL);
    switch (ks) {
    case XK_Escape: fprintf(stderr, "Done.\n"); return 0;
    case XK_Up: key(h, 'U'); return 1;
    case XK_Down: key(h, 'D'); return 1;
    case XK_Left: key(h, 'L'); return 1;
    case XK_Right: key(h, 'R'); return 1;
    case XK_Page_Up: key(h, 'P'); return 1;
    case XK_Page_Down: key(h, 'Q'); return 1;
    default: break;
    }
    if (n != 1) return 1;
    const int c = (unsigned char)buf[0];
    if (c == 'h') {
        v->print_help = !v->print_help;
    } else if (c == 'i') {
        printf("Origin:(%.1f,%.1f,%.1f)\n\nTarget:(%.1f,%.1f,%.1f)", h->camera.orig.x, h->camera.orig.y,
               h->camera.orig.z, h->camera.target.x, h->camera.target.y, h->camera.target.z);
    } else if (strchr("pad wsrf+-468293", c)) {  /* KeyFunc's keys ('5' is listed in the help only) */
        key(h, c);
    }
    return 1;
}

int main(int argc, char **argv)
{
    host h;
    view v;
    memset(&h, 0, sizeof h);
    memset(&v, 0, sizeof v);
    v.print_help = 1;                             /* display_func.c:58 */
    int device = 0, batch = 1, npos = 0;
    long frames = 0;
    const char *pos[3] = {0, 0, 0}, *dat = "assets/data/MersenneTwister.dat";
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "--device") && a + 1 < argc) device = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--batch") && a + 1 < argc) batch = atoi(argv[++a]);
        else if (!strcmp(argv[a], "--frames") && a + 1 < argc) frames = atol(argv[++a]);
        else if (!strcmp(argv[a], "--dat") && a + 1 < argc) dat = argv[++a];
        else if (npos < 3) pos[npos++] = argv[a];
        else { fprintf(stderr, "Usage: %s <window width> <window height> <scene file>\n", argv[0]); return -1; }
    }
    if (batch < 1) batch = 1;
    if (npos == 3) {
        h.width = atoi(pos[0]);
        h.height = atoi(pos[1]);
        fprintf(stderr, "Reading scene: %s\n", pos[2]);
        if (bdpt_read_scene(pos[2], &h.camera, &h.spheres, &h.n) != BDPT_OK) exit(-1);
    } else if (npos == 0) {
        h.width = 640;
        h.height = 480;
        h.spheres = malloc(sizeof(bdpt_sphere) * 9);
        h.n = bdpt_default_scene(&h.camera, h.spheres);
    } else {
        exit(-1);
    }
    h.height += 1;                                /* smallpt_cpu.c:409-410 */
    h.width += 1;
    bdpt_update_camera(&h.camera, h.width, h.height);
    bdpt_pass_state_init(&h.ps);

    /* InitGlut: the window and its GL context come first, before any GPU work */
    v.dpy = XOpenDisplay(NULL);
    if (!v.dpy) {
        const char *d = getenv("DISPLAY");
        fprintf(stderr, "smallpt_gl: cannot open X display '%s'\n", d ? d : "");
        if (npos == 3) bdpt_free_scene(h.spheres); else free(h.spheres);
        return 2;
    }
    int attr[] = {GLX_RGBA, GLX_DOUBLEBUFFER, GLX_RED_SIZE, 8, GLX_GREEN_SIZE, 8, GLX_BLUE_SIZE, 8, None};
    XVisualInfo *vi = glXChooseVisual(v.dpy, DefaultScreen(v.dpy), attr);
    if (!vi) {
        fprintf(stderr, "smallpt_gl: no double-buffered RGBA visual\n");
        XCloseDisplay(v.dpy);
        return 2;
    }
    XSetWindowAttributes swa;
    memset(&swa, 0, sizeof swa);
    swa.colormap = XCreateColormap(v.dpy, RootWindow(v.dpy, vi->screen), vi->visual, AllocNone);
    swa.event_mask = KeyPressMask | ExposureMask | StructureNotifyMask;
    v.win = XCreateWindow(v.dpy, RootWindow(v.dpy, vi->screen), 0, 0, (unsigned)h.width, (unsigned)h.height, 0,
                          vi->depth, InputOutput, vi->visual, CWColormap | CWEventMask, &swa);
    XStoreName(v.dpy, v.win, "DR");               /* InitGlut(argc, argv, "DR") smallpt_cpu.c:418 */
    Atom wm_delete = XInternAtom(v.dpy, "WM_DELETE_WINDOW", False);
    XSetWMProtocols(v.dpy, v.win, &wm_delete, 1);
    XMapWindow(v.dpy, v.win);
    v.glc = glXCreateContext(v.dpy, vi, NULL, True);
    XFree(vi);
    if (!v.glc || !glXMakeCurrent(v.dpy, v.win, v.glc)) {
        fprintf(stderr, "smallpt_gl: cannot create a GLX context\n");
        XCloseDisplay(v.dpy);
        return 2;
    }
    XFontStruct *fs = XLoadQueryFont(v.dpy, "fixed");
    if (fs) {
        v.font = glGenLists(96);
        glXUseXFont(fs->fid, 32, 96, v.font);
    }
    reshape(h.width, h.height);

    /* createPBO / createTexture smallpt_cpu.c:112-140 */
    glGenBuffers(1, &v.pbo);
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, v.pbo);
    glBufferData(GL_PIXEL_UNPACK_BUFFER, 4 * (GLsizeiptr)h.width * h.height, NULL, GL_DYNAMIC_COPY);
    glBindBuffer(GL_PIXEL_UNPACK_BUFFER, 0);
    glEnable(GL_TEXTURE_2D);
    glGenTextures(1, &v.tex);
    glBindTexture(GL_TEXTURE_2D, v.tex);
    glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MIN_FILTER, GL_NEAREST);
    glTexParameteri(GL_TEXTURE_2D, GL_TEXTURE_MAG_FILTER, GL_NEAREST);
    glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA8, h.width, h.height, 0, GL_RGBA, GL_UNSIGNED_BYTE, NULL);

    fprintf(stderr, "Allocate Buffers\n");
    int rc = bdpt_create(&h.ctx, h.spheres, h.n, h.width, h.height, dat, device);
    if (rc != BDPT_OK) {
        fprintf(stderr, "Unable to allocate GPU data: %s\n", bdpt_create_error());
    } else {
        report(&h, rc = bdpt_set_camera(h.ctx, &h.camera), "camera");
        if (rc == BDPT_OK) report(&h, rc = bdpt_gl_register_pbo(h.ctx, v.pbo), "Register Buffer");
    }
    if (rc == BDPT_OK) {
        update_rendering2(&h);                    /* IdleFunc, flag == 1 */
        int run = 1;
        for (long shown = 0; run;) {
            while (XPending(v.dpy)) {
                XEvent ev;
                XNextEvent(v.dpy, &ev);
                if (ev.type == ConfigureNotify) reshape(ev.xconfigure.width, ev.xconfigure.height);
                else if (ev.type == KeyPress) run = run && on_key(&v, &h, &ev.xkey);
                else if (ev.type == ClientMessage && (Atom)ev.xclient.data.l[0] == wm_delete) run = 0;
            }
            if (!run) break;
            update_rendering(&h, batch);          /* IdleFunc, flag > 1 */
            rc = bdpt_gl_publish(h.ctx);
            report(&h, rc, "Map Buffer");
            if (rc != BDPT_OK) break;
            display(&v, &h);
            if (frames > 0 && ++shown >= frames) break;
        }
        report(&h, bdpt_gl_unregister(h.ctx), "Unregister Buffer");
    }
    bdpt_destroy(h.ctx);
    glDeleteTextures(1, &v.tex);
    glDeleteBuffers(1, &v.pbo);
    if (v.font) glDeleteLists(v.font, 96);
    if (fs) XFreeFont(v.dpy, fs);
    glXMakeCurrent(v.dpy, None, NULL);
    glXDestroyContext(v.dpy, v.glc);
    XDestroyWindow(v.dpy, v.win);
    XCloseDisplay(v.dpy);
    if (npos == 3) bdpt_free_scene(h.spheres); else free(h.spheres);
    return rc == BDPT_OK ? 0 : 1;
}
