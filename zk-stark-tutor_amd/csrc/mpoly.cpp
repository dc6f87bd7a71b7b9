// placeholder (filled below)
