// USB stereo camera capture over V4L2 (reference usb_test.py:7-35: 1280x480 MJPG at 30 fps from
// /dev/video0, 'k' saves <i>.jpg, 'q' quits).  Headless: frames are saved on a key read from
// stdin ('k' + Enter saves the next frame, 'q' + Enter quits) or every --every N frames; --split
// also writes left<i>.jpg / right<i>.jpg halves (Stereo_Calibration/process_image.py).  MJPG
// frames are decoded with the framework's own baseline JPEG codec; YUYV cameras are converted.
//
//   stereo_capture [--device /dev/video0] [--width 1280] [--height 480] [--fps 30]
//                  [--every N] [--count N] [--split] [--out DIR]
#include <fcntl.h>
#include <linux/videodev2.h>
#include <poll.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sa/imgio.h"
#include "sa/mat.h"

namespace {

int xioctl(int fd, unsigned long req, void* arg) {
  int r;
  do r = ioctl(fd, req, arg);
  while (r == -1 && errno == EINTR);
  return r;
}

unsigned char clamp8(int v) { return (unsigned char)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// YUYV 4:2:2 -> BGR (BT.601 limited range, as V4L2 cameras deliver it)
void yuyv_to_bgr(const unsigned char* src, int w, int h, unsigned char* dst) {
  for (int i = 0; i < w * h / 2; ++i) {
    const int y0 = src[4 * i] - 16, u = src[4 * i + 1] - 128, y1 = src[4 * i + 2] - 16, v = src[4 * i + 3] - 128;
    for (int k = 0; k < 2; ++k) {
      const int c = 298 * (k ? y1 : y0);
      unsigned char* o = dst + 6 * i + 3 * k;
      o[0] = clamp8((c + 516 * u + 128) >> 8);
      o[1] = clamp8((c - 100 * u - 208 * v + 128) >> 8);
      o[2] = clamp8((c + 409 * v + 128) >> 8);
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::string dev = "/dev/video0", out = ".";
  int width = 1280, height = 480, fps = 30, every = 0, count = -1;
  bool split = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (a == "--device") dev = next();
    else if (a == "--width") width = std::atoi(next().c_str());
    else if (a == "--height") height = std::atoi(next().c_str());
    else if (a == "--fps") fps = std::atoi(next().c_str());
    else if (a == "--every") every = std::atoi(next().c_str());
    else if (a == "--count") count = std::atoi(next().c_str());
    else if (a == "--split") split = true;
    else if (a == "--out") out = next();
    else {
      std::printf("usage: %s [--device /dev/video0] [--width 1280] [--height 480] [--fps 30] [--every N] "
                  "[--count N] [--split] [--out DIR]\n", argv[0]);
      return a == "-h" || a == "--help" ? 0 : 2;
    }
  }
  const int fd = open(dev.c_str(), O_RDWR | O_NONBLOCK);
  if (fd < 0) {
    std::fprintf(stderr, "cannot open %s: %s\n", dev.c_str(), std::strerror(errno));
    return 1;
  }
  v4l2_format fmt{};
  fmt.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
  fmt.fmt.pix.width = width;
  fmt.fmt.pix.height = height;
  fmt.fmt.pix.pixelformat = V4L2_PIX_FMT_MJPEG;
  fmt.fmt.pix.field = V4L2_FIELD_ANY;
  if (xioctl(fd, VIDIOC_S_FMT, &fmt) < 0) {
    fmt.fmt.pix.pixelformat = V4L2_PIX_FMT_YUYV;
    if (xioctl(fd, VIDIOC_S_FMT, &fmt) < 0) {
      std::fprintf(stderr, "VIDIOC_S_FMT failed: %s\n", std::strerror(errno));
      return 1;
    }
  }
  width = fmt.fmt.pix.width;
  height = fmt.fmt.pix.height;
  const bool mjpg = fmt.fmt.pix.pixelformat == V4L2_PIX_FMT_MJPEG;
  v4l2_streamparm parm{};
  parm.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
  parm.parm.capture.timeperframe.numerator = 1;
  parm.parm.capture.timeperframe.denominator = fps;
  (void)xioctl(fd, VIDIOC_S_PARM, &parm);  // best effort, as cap.set(CAP_PROP_FPS)

  v4l2_requestbuffers req{};
  req.count = 4;
  req.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
  req.memory = V4L2_MEMORY_MMAP;
  if (xioctl(fd, VIDIOC_REQBUFS, &req) < 0 || req.count < 2) {
    std::fprintf(stderr, "VIDIOC_REQBUFS failed\n");
    return 1;
  }
  std::vector<void*> bufs(req.count);
  std::vector<size_t> lens(req.count);
  for (unsigned i = 0; i < req.count; ++i) {
    v4l2_buffer b{};
    b.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
    b.memory = V4L2_MEMORY_MMAP;
    b.index = i;
    if (xioctl(fd, VIDIOC_QUERYBUF, &b) < 0) return 1;
    lens[i] = b.length;
    bufs[i] = mmap(nullptr, b.length, PROT_READ | PROT_WRITE, MAP_SHARED, fd, b.m.offset);
    if (bufs[i] == MAP_FAILED) return 1;
    if (xioctl(fd, VIDIOC_QBUF, &b) < 0) return 1;
  }
  v4l2_buf_type type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
  if (xioctl(fd, VIDIOC_STREAMON, &type) < 0) {
    std::fprintf(stderr, "VIDIOC_STREAMON failed: %s\n", std::strerror(errno));
    return 1;
  }
  std::printf("capturing %dx%d %s from %s; enter k to save, q to exit\n", width, height, mjpg ? "MJPG" : "YUYV",
              dev.c_str());
  int saved = 0;
  long frame = 0;
  bool save_next = false, quit = false;
  std::vector<unsigned char> bgr((size_t)width * height * 3);
  while (!quit && (count < 0 || saved < count)) {
    pollfd pf[2] = {{fd, POLLIN, 0}, {0, POLLIN, 0}};
    if (poll(pf, every > 0 ? 1 : 2, 2000) <= 0) continue;
    if (every <= 0 && (pf[1].revents & POLLIN)) {
      char line[64];
      if (!std::fgets(line, sizeof(line), stdin)) break;
      if (line[0] == 'q') quit = true;
      if (line[0] == 'k') save_next = true;
    }
    if (!(pf[0].revents & POLLIN)) continue;
    v4l2_buffer b{};
    b.type = V4L2_BUF_TYPE_VIDEO_CAPTURE;
    b.memory = V4L2_MEMORY_MMAP;
    if (xioctl(fd, VIDIOC_DQBUF, &b) < 0) continue;
    ++frame;
    const bool save = save_next || (every > 0 && frame % every == 0);
    if (save) {
      sa::Mat img;
      bool ok = true;
      if (mjpg) {
        sa::Image im;
        ok = sa::jpeg_decode(static_cast<const uint8_t*>(bufs[b.index]), b.bytesused, im) && im.channels == 3;
        if (ok) img = sa::Mat(im.height, im.width, sa::SA_8UC3, im.data.data()).clone();
      } else {
        yuyv_to_bgr(static_cast<const unsigned char*>(bufs[b.index]), width, height, bgr.data());
        img = sa::Mat(height, width, sa::SA_8UC3, bgr.data()).clone();
      }
      if (ok) {
        const std::string name = out + "/" + std::to_string(saved) + ".jpg";
        sa::imwrite(name, img);
        if (split) {
          const int wl = img.cols / 2;
          sa::Mat l(img.rows, wl, sa::SA_8UC3, img.data, img.step), r(img.rows, img.cols - wl, sa::SA_8UC3,
                                                                        img.data + (size_t)wl * 3, img.step);
          sa::imwrite(out + "/left" + std::to_string(saved) + ".jpg", l.clone());
          sa::imwrite(out + "/right" + std::to_string(saved) + ".jpg", r.clone());
        }
        std::printf("the %d image saved!\n", saved);
        ++saved;
      }
      save_next = false;
    }
    (void)xioctl(fd, VIDIOC_QBUF, &b);
  }
  (void)xioctl(fd, VIDIOC_STREAMOFF, &type);
  for (unsigned i = 0; i < req.count; ++i) munmap(bufs[i], lens[i]);
  close(fd);
  return 0;
}
