"""Flow set-ups: turbulent channel (ChannelFlow), laminar Poiseuille, Orr-Sommerfeld modes."""
